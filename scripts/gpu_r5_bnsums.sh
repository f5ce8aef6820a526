#!/bin/bash
# round 5: block-output BN applied from the epilogue sums (no finalize
# dispatch) -- engine / BN tests, same-tiles A/B of the graphed forward,
# forward breakdown at 1 clip (dispatch count)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
trace_of() { ls $1/*/*/run_kernel_trace.csv $1/*/run_kernel_trace.csv $1/run_kernel_trace.csv 2>/dev/null | tail -1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_f32.py -x -q --timeout 120 --timeout-method thread \
  -k "apply_from_sums or batched_running or bn_ or graphed or top1 or running" > gpurun_out/bnsums_tests.log 2>&1 || { tail -40 gpurun_out/bnsums_tests.log; exit 1; }
tail -3 gpurun_out/bnsums_tests.log
timeout -k 10 500 python scripts/graph_ab.py --env RNB_BN_SS_ONLY --a 0 --b 1 --clips 128 16 1 > gpurun_out/graph_ab_ss_only.txt 2>&1 || { tail gpurun_out/graph_ab_ss_only.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/graph_ab_ss_only.txt
d=gpurun_out/bnb_1; rm -rf $d
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
  -- python3 scripts/bn_breakdown.py run --mode batch --clips 1 > $d.log 2>&1 || { echo "bnb 1 failed"; tail $d.log; exit 1; }
python3 scripts/bn_breakdown.py parse "$(trace_of $d)" --kernels 14 > gpurun_out/bnb_1.txt
head -16 gpurun_out/bnb_1.txt
rm -rf $d
