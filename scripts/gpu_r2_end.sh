#!/bin/bash
# Round-end style check of the final tree: full GPU suite, smoke, default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/end2_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/end2_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/end2_smoke.log 2>&1
rc=$?; grep smoke gpurun_out/end2_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 2 --json-out gpurun_out/end2_bench.json \
  > gpurun_out/end2_bench.log 2>&1
rc=$?; grep -E "Throughput|Latency phase" gpurun_out/end2_bench.log; exit $rc
