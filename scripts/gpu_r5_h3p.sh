#!/bin/bash
# round 5: pixel-major temporal h3 kernel (conv_h3p) -- its tests, then the
# conv2 / stem temporal layer table against h3t
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_h3.py -x -v --timeout 120 --timeout-method thread \
  -k "h3p or (temporal_band and h3t)" > gpurun_out/h3p_tests.log 2>&1 || { tail -60 gpurun_out/h3p_tests.log; exit 1; }
tail -3 gpurun_out/h3p_tests.log
timeout -k 10 300 python scripts/h3_layer_bench.py --clips 128 --cases k4,stemt,stemt45 --only-h3 > gpurun_out/h3p_layers.txt 2>&1 || { tail gpurun_out/h3p_layers.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/h3p_layers.txt | head -40
