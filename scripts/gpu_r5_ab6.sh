#!/bin/bash
# round 5: why geometric buckets make smaller bulk calls -- bucket-fit trimming
# off (RNB_FIT_PAD_FRAC=1) against the default and 4-clip buckets, 20 steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python scripts/ab_bench.py --rounds 2 --out gpurun_out/ab_fit.txt \
  "geo||--steps 20" "geonofit|RNB_FIT_PAD_FRAC=1|--steps 20" "step4||--steps 20 --bucket-step 4"
rc=$?; cat gpurun_out/ab_fit.txt; exit $rc
