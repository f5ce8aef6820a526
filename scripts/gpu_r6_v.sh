#!/bin/bash
# round 6: block-tiled BN apply -- GPU tests, then graphed-forward wall time
# per bucket with the block-tiled vs the per-thread-row applies (interleaved),
# then a kernel table at 128 clips
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_bn_apply.py tests/test_gpu_engine.py -k "apply or batch or sums or running or blocked" \
  > gpurun_out/v_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/v_tests.log; exit 1; }
tail -3 gpurun_out/v_tests.log
out=gpurun_out/ab_apply.txt; : > $out
for rnd in 1 2; do
  for c in 128 16 1; do
    for b in 0 1; do
      r=$(RNB_BN_APPLY_BLK=$b timeout -k 10 300 python3 scripts/bn_breakdown.py run --mode batch --clips $c --reps 30 2>&1 | tail -1) || { echo "run failed: $r"; exit 1; }
      echo "round $rnd clips $c apply_blk $b: $r" | tee -a $out
    done
  done
done
trace_of() { ls $1/*/*/run_kernel_trace.csv $1/*/run_kernel_trace.csv $1/run_kernel_trace.csv 2>/dev/null | tail -1; }
d=gpurun_out/bnbv_128; rm -rf $d
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
  -- python3 scripts/bn_breakdown.py run --mode batch --clips 128 > $d.log 2>&1 || { echo "bnb failed"; tail $d.log; exit 1; }
python3 scripts/bn_breakdown.py parse "$(trace_of $d)" --kernels 16 > gpurun_out/bnbv_128.txt
head -30 gpurun_out/bnbv_128.txt
rm -rf $d
