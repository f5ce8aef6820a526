#!/bin/bash
# round 5: wave-specialised temporal kernel (conv_h3u): correctness, layer timing, bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_h3.py -k "temporal_band" -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_h3u.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_h3u.log | tail -40
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/h3_layer_bench.py --clips 128 --cases k4,k8,k14 --only-h3 > gpurun_out/layers_h3u.txt 2>&1
rc=$?; head -12 gpurun_out/layers_h3u.txt; grep -E "cid 14" gpurun_out/layers_h3u.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --json-out gpurun_out/bench_h3u.json > gpurun_out/bench_h3u.log 2>&1
rc=$?; tail -c 600 gpurun_out/bench_h3u.log; exit $rc
