#!/bin/bash
# round 6: 224-pixel row-band h3r variant with two blocks per CU (id 1389)
# against the row-band picks on the spatial convs, then its GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_h3.py -k "rowband" > gpurun_out/aa_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/aa_tests.log; exit 1; }
tail -2 gpurun_out/aa_tests.log
timeout -k 10 500 python3 scripts/h3_layer_bench.py --clips 128 --cases k3,k3a,k7,k7a,k13,k13a \
  --cids 1380,1381,1382,1383,1384,1385,1386,1387,1388,1389 --rounds 2 > gpurun_out/aa_layers_128.txt 2>&1 || { tail gpurun_out/aa_layers_128.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/aa_layers_128.txt | awk '{print $1, $4, $5}' | head -70
timeout -k 10 300 python3 scripts/h3_layer_bench.py --clips 16 --cases k3,k3a,k7,k7a \
  --cids 1380,1383,1386,1387,1388,1389,1461 --rounds 2 > gpurun_out/aa_layers_16.txt 2>&1 || { tail gpurun_out/aa_layers_16.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/aa_layers_16.txt | awk '{print $1, $4, $5}'
