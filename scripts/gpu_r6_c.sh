#!/bin/bash
# round 6: Poisson tail A/B -- the 1-clip-video replicas on CU-masked streams
# (3/4 and 1/2 of the CUs) so 15-clip calls find CUs free; longer latency
# phases for a steadier p99
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u -m pytest tests/test_gpu_cumask.py -q -p no:cacheprovider --timeout 60 --timeout-method thread > gpurun_out/cumask_test.log 2>&1
rc=$?; tail -3 gpurun_out/cumask_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1500 python scripts/ab_bench.py --rounds 2 --steps 10 --timeout 300 \
  --out gpurun_out/ab_cumask.txt \
  "base||--latency-seconds 6" "cu75||--latency-seconds 6 --small-cu-frac 0.75" \
  "cu50||--latency-seconds 6 --small-cu-frac 0.5"
