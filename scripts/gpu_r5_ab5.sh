#!/bin/bash
# round 5: headline regression check -- geometric vs 4-clip graph buckets, and
# the h3 range guard off, interleaved at 20 steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python scripts/ab_bench.py --rounds 2 --out gpurun_out/ab_geo20.txt \
  "geo||--steps 20" "step4||--steps 20 --bucket-step 4" "noguard|RNB_H3_GUARD=0|--steps 20"
rc=$?; cat gpurun_out/ab_geo20.txt; exit $rc
