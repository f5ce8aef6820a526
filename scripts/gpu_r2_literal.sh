#!/bin/bash
# Literal benchmark.py runs with the runner's default BatchNorm numerics
# (batch statistics at fp32, the reference's): the reference rnb topology at
# saturation, and the reference's published setup (r2p1d-whole, R(2+1)D-18,
# 500 videos, Poisson 90 ms).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 RNB_NO_TQDM=1
timeout -k 10 400 python benchmark.py -c configs/rnb-1gpu.json -mi 0 -v 3000 --warmup-videos 500 \
  --json-out gpurun_out/lit_rnb1gpu.json > gpurun_out/lit_rnb1gpu.log 2>&1
rc=$?; echo "=== rnb-1gpu rc=$rc"; grep -E "Throughput|latency over|batched calls" gpurun_out/lit_rnb1gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python benchmark.py -c configs/r2p1d-whole-r18.json -mi 90 -v 500 \
  --json-out gpurun_out/lit_whole_r18.json > gpurun_out/lit_whole_r18.log 2>&1
rc=$?; echo "=== whole-r18 rc=$rc"; grep -E "Throughput|latency over|Average time" gpurun_out/lit_whole_r18.log
exit $rc
