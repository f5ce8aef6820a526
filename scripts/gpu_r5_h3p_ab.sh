#!/bin/bash
# round 5: pixel-major temporal h3 kernel in the graphed forward -- tests,
# separately tuned A/B (RNB_H3P 0 / 1), forward breakdown at 128 clips
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
trace_of() { ls $1/*/*/run_kernel_trace.csv $1/*/run_kernel_trace.csv $1/run_kernel_trace.csv 2>/dev/null | tail -1; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_h3.py -x -q --timeout 120 --timeout-method thread \
  -k "h3p or temporal_band" > gpurun_out/h3p_tests.log 2>&1 || { tail -40 gpurun_out/h3p_tests.log; exit 1; }
tail -2 gpurun_out/h3p_tests.log
timeout -k 10 600 python scripts/graph_ab.py --env RNB_H3P --a 0 --b 1 --retune --clips 128 16 > gpurun_out/graph_ab_h3p.txt 2>&1 || { tail gpurun_out/graph_ab_h3p.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/graph_ab_h3p.txt
d=gpurun_out/bnb_128; rm -rf $d
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
  -- python3 scripts/bn_breakdown.py run --mode batch --clips 128 > $d.log 2>&1 || { echo "bnb 128 failed"; tail $d.log; exit 1; }
python3 scripts/bn_breakdown.py parse "$(trace_of $d)" --kernels 16 > gpurun_out/bnb_128_h3p.txt
head -32 gpurun_out/bnb_128_h3p.txt
rm -rf $d
