#!/bin/bash
# Fused BN finalize (<= 32 segments): BN tests + 24 / 32 / 128-clip breakdown A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 RNB_TUNE_CACHE=$PWD/gpurun_out/tune_fr2.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py -k "bn" -x -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/fr2_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/fr2_tests.log; [ $rc -eq 0 ] || exit $rc
for clips in 24 32 128; do
for mode in 1 0; do
  name="bnb_fr2_${mode}_${clips}"
  rm -rf "gpurun_out/$name"
  RNB_BN_FUSED_FINALIZE=$mode timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv \
    -d "gpurun_out/$name" -o run -- python3 scripts/bn_breakdown.py run --mode batch --clips $clips \
    > "gpurun_out/$name.log" 2>&1
  rc=$?; echo "=== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
  trace=$(ls gpurun_out/$name/*/*/run_kernel_trace.csv gpurun_out/$name/*/run_kernel_trace.csv gpurun_out/$name/run_kernel_trace.csv 2>/dev/null | tail -1)
  python3 scripts/bn_breakdown.py parse "$trace" --kernels 6 > "gpurun_out/$name.txt"
  head -n 9 "gpurun_out/$name.txt"
  rm -rf "gpurun_out/$name"
done
done
