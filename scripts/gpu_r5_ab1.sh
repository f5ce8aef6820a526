#!/bin/bash
# round 5: geo vs 4-clip graph buckets (interleaved A/B) + temporal-conv layer table
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python scripts/h3_layer_bench.py --clips 128 --cases k4,k4c128,k4c160,k8,k14 --only-h3 > gpurun_out/layers_temporal.txt 2>&1
rc=$?; tail -40 gpurun_out/layers_temporal.txt; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 840 python scripts/ab_bench.py --rounds 2 --out gpurun_out/ab_geo.txt \
  "geo||--steps 10" "s4||--steps 10 --bucket-step 4"
rc=$?; cat gpurun_out/ab_geo.txt; exit $rc
