#!/bin/bash
# round 5: lanes of the 15-clip-video replica (2 default vs 3), 20 steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python scripts/ab_bench.py --rounds 2 --out gpurun_out/ab_large_lanes3.txt \
  "ll2||--steps 20" "ll3||--steps 20 --large-lanes 3"
rc=$?; cat gpurun_out/ab_large_lanes3.txt; exit $rc
