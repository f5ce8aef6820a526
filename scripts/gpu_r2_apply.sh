#!/bin/bash
# Streaming BN apply: kernel tests, kernel-family breakdown of the graphed
# batch-BN forward with the streaming vs the row-loop apply, then the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py -k "bn_" -x -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/apply_tests.log 2>&1
rc=$?; tail -n 12 gpurun_out/apply_tests.log; [ $rc -eq 0 ] || exit $rc
for mode in 1 0; do
  name="bnb_apply${mode}_128"
  rm -rf "gpurun_out/$name"
  RNB_BN_APPLY_STREAM=$mode timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv \
    -d "gpurun_out/$name" -o run -- python3 scripts/bn_breakdown.py run --mode batch --clips 128 \
    > "gpurun_out/$name.log" 2>&1
  rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
  trace=$(ls gpurun_out/$name/*/*/run_kernel_trace.csv gpurun_out/$name/*/run_kernel_trace.csv gpurun_out/$name/run_kernel_trace.csv 2>/dev/null | tail -1)
  python3 scripts/bn_breakdown.py parse "$trace" --kernels 12 | tee "gpurun_out/$name.txt"
  rm -rf "gpurun_out/$name"
done
timeout -k 10 600 python bench.py --steps 20 --warmup 2 --json-out gpurun_out/bench_apply.json \
  > gpurun_out/bench_apply.log 2>&1
rc=$?; tail -n 3 gpurun_out/bench_apply.log; exit $rc
