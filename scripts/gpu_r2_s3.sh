#!/bin/bash
# Session-3 check: full GPU suite, kernel-family breakdown of the graphed
# batch-BN forward (128 clips), headline bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/s3_pytest.log 2>&1
rc=$?; tail -n 4 gpurun_out/s3_pytest.log; [ $rc -eq 0 ] || exit $rc
name=bnb_s3_128
rm -rf "gpurun_out/$name"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "gpurun_out/$name" -o run -- \
  python3 scripts/bn_breakdown.py run --mode batch --clips 128 > "gpurun_out/$name.log" 2>&1
rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
trace=$(ls gpurun_out/$name/*/*/run_kernel_trace.csv gpurun_out/$name/*/run_kernel_trace.csv gpurun_out/$name/run_kernel_trace.csv 2>/dev/null | tail -1)
python3 scripts/bn_breakdown.py parse "$trace" --kernels 14 | tee "gpurun_out/$name.txt"
rm -rf "gpurun_out/$name"
timeout -k 10 600 python bench.py --steps 20 --warmup 2 --json-out gpurun_out/bench_s3.json \
  > gpurun_out/bench_s3.log 2>&1
rc=$?; tail -n 3 gpurun_out/bench_s3.log; exit $rc
