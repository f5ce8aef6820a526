#!/bin/bash
# round 5: stem h3 kernel (conv_h3stem) -- its tests and the stem layer table
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_h3.py -x -q --timeout 120 --timeout-method thread \
  -k "h3stem or stem_exact" > gpurun_out/stem_tests.log 2>&1 || { tail -40 gpurun_out/stem_tests.log; exit 1; }
tail -3 gpurun_out/stem_tests.log
timeout -k 10 300 python scripts/h3_layer_bench.py --clips 128 --cases stem > gpurun_out/stem_layers2.txt 2>&1 || { tail gpurun_out/stem_layers2.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stem_layers2.txt | head -12
