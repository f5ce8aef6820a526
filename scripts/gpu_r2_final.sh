#!/bin/bash
# End-of-session check: full GPU suite, smoke, fused-finalize A/B breakdown
# (24 / 128 clips), default bench (20 steps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/final_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/final_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1
rc=$?; grep smoke gpurun_out/final_smoke.log; [ $rc -eq 0 ] || exit $rc
export RNB_TUNE_CACHE=$PWD/gpurun_out/tune_final.json
for clips in 24 128; do
for mode in 1 0; do
  name="bnb_final_fr${mode}_${clips}"
  rm -rf "gpurun_out/$name"
  RNB_BN_FUSED_FINALIZE=$mode timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv \
    -d "gpurun_out/$name" -o run -- python3 scripts/bn_breakdown.py run --mode batch --clips $clips \
    > "gpurun_out/$name.log" 2>&1
  rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
  trace=$(ls gpurun_out/$name/*/*/run_kernel_trace.csv gpurun_out/$name/*/run_kernel_trace.csv gpurun_out/$name/run_kernel_trace.csv 2>/dev/null | tail -1)
  python3 scripts/bn_breakdown.py parse "$trace" --kernels 6 > "gpurun_out/$name.txt"
  head -n 10 "gpurun_out/$name.txt"
  rm -rf "gpurun_out/$name"
done
done
unset RNB_TUNE_CACHE
timeout -k 10 600 python bench.py --steps 20 --warmup 2 --json-out gpurun_out/final_bench.json \
  > gpurun_out/final_bench.log 2>&1
rc=$?; grep -E "Throughput|Latency phase" gpurun_out/final_bench.log; tail -n 1 gpurun_out/final_bench.log | cut -c1-400
exit $rc
