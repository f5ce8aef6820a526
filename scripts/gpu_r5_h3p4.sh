#!/bin/bash
# round 5: the pixel-major temporal kernel's 4-frame form (conv3 temporal,
# 32-channel slices, 2 tiles per task) -- tests, then k8 / k4 / stem temporal
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_h3.py -x -v --timeout 120 --timeout-method thread \
  -k "h3p or temporal_band" > gpurun_out/h3p4_tests.log 2>&1 || { tail -50 gpurun_out/h3p4_tests.log; exit 1; }
tail -2 gpurun_out/h3p4_tests.log
timeout -k 10 300 python scripts/h3_layer_bench.py --clips 128 --cases k8,k4,stemt --only-h3 > gpurun_out/h3p4_layers.txt 2>&1 || { tail gpurun_out/h3p4_layers.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/h3p4_layers.txt | awk '{c[$1]++} c[$1] <= 5'
