#!/bin/bash
# round 6: split-K reduce with one row per thread for small outputs -- graphed
# forward wall time at 1 / 4 / 16 clips against the old 4 rows per thread
# (interleaved), the split-K GPU tests, and a 1-clip kernel table
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_h3.py tests/test_gpu_f32.py -k "splitk or split" > gpurun_out/ae_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ae_tests.log; exit 1; }
tail -2 gpurun_out/ae_tests.log
out=gpurun_out/ab_splitk_rpt.txt; : > $out
for rnd in 1 2; do
  for c in 1 4 16; do
    for r in 4 0; do
      v=$(RNB_SPLITK_RPT=$r timeout -k 10 200 python3 scripts/bn_breakdown.py run --mode batch --clips $c --reps 200 2>&1 | tail -1) || { echo "run failed: $v"; exit 1; }
      echo "round $rnd clips $c rpt ${r/0/auto}: $v" | tee -a $out
    done
  done
done
trace_of() { ls $1/*/*/run_kernel_trace.csv $1/*/run_kernel_trace.csv $1/run_kernel_trace.csv 2>/dev/null | tail -1; }
d=gpurun_out/bnbe_1; rm -rf $d
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
  -- python3 scripts/bn_breakdown.py run --mode batch --clips 1 > $d.log 2>&1 || { echo "bnb failed"; tail $d.log; exit 1; }
python3 scripts/bn_breakdown.py parse "$(trace_of $d)" --kernels 12 > gpurun_out/bnbe_1.txt
head -16 gpurun_out/bnbe_1.txt
rm -rf $d
