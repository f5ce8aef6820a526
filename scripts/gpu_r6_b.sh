#!/bin/bash
# round 6: graph-bucket spacing A/B with the seed table on (geo = geometric,
# geo8 = geometric below 96 clips then every 8, s4 = every 4 clips, nofit =
# geo without the bucket-fit trim), interleaved rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1500 python scripts/ab_bench.py --rounds 2 --steps 10 --timeout 300 \
  --out gpurun_out/ab_buckets.txt \
  "geo||" "geo8||--bucket-step geo8" "s4||--bucket-step 4" "nofit|RNB_FIT_PAD_FRAC=1|"
