#!/bin/bash
# round 6: consumer-side input BN rows (h3 direct computes its scale / shift
# from the producer's sums): tests, then graphed forward wall time at 1 / 4 /
# 16 clips against the finalize dispatches (interleaved), and a 1-clip table
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_bn_tail.py -k "sums" > gpurun_out/af_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/af_tests.log; exit 1; }
tail -2 gpurun_out/af_tests.log
out=gpurun_out/ab_aff_sums.txt; : > $out
for rnd in 1 2; do
  for c in 1 4 16; do
    for m in 0 2304; do
      v=$(RNB_BN_AFF_SUMS_MAX=$m timeout -k 10 200 python3 scripts/bn_breakdown.py run --mode batch --clips $c --reps 200 2>&1 | tail -1) || { echo "run failed: $v"; exit 1; }
      echo "round $rnd clips $c aff_sums_max $m: $v" | tee -a $out
    done
  done
done
trace_of() { ls $1/*/*/run_kernel_trace.csv $1/*/run_kernel_trace.csv $1/run_kernel_trace.csv 2>/dev/null | tail -1; }
d=gpurun_out/bnbg_1; rm -rf $d
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
  -- python3 scripts/bn_breakdown.py run --mode batch --clips 1 > $d.log 2>&1 || { echo "bnb failed"; tail $d.log; exit 1; }
python3 scripts/bn_breakdown.py parse "$(trace_of $d)" --kernels 12 > gpurun_out/bnbg_1.txt
head -16 gpurun_out/bnbg_1.txt
rm -rf $d
