#!/bin/bash
# round 5: h3t bottleneck attribution, then the Poisson-tail A/B (small replicas
# yield to a running 15-clip call in the latency regime)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python scripts/ab_bench.py --rounds 2 --out gpurun_out/ab_yield.txt \
  "base||--steps 10" "y4||--steps 10 --yield-ms 4" "y8||--steps 10 --yield-ms 8"
rc=$?; cat gpurun_out/ab_yield.txt; exit $rc
