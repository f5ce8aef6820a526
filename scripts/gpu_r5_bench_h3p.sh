#!/bin/bash
# round 5: bench with the pixel-major temporal kernel -- driver defaults,
# then 20 steps; the 1-clip forward breakdown (dispatch count)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
trace_of() { ls $1/*/*/run_kernel_trace.csv $1/*/run_kernel_trace.csv $1/run_kernel_trace.csv 2>/dev/null | tail -1; }
timeout -k 10 560 python bench.py --json-out gpurun_out/bench_h3p_default.json > gpurun_out/bench_h3p_default.log 2>&1 || { tail gpurun_out/bench_h3p_default.log; exit 1; }
tail -1 gpurun_out/bench_h3p_default.log
timeout -k 10 560 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_h3p_20.json > gpurun_out/bench_h3p_20.log 2>&1 || { tail gpurun_out/bench_h3p_20.log; exit 1; }
tail -1 gpurun_out/bench_h3p_20.log
d=gpurun_out/bnb_1; rm -rf $d
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
  -- python3 scripts/bn_breakdown.py run --mode batch --clips 1 > $d.log 2>&1 || { echo "bnb 1 failed"; tail $d.log; exit 1; }
python3 scripts/bn_breakdown.py parse "$(trace_of $d)" --kernels 14 > gpurun_out/bnb_1_h3p.txt
head -14 gpurun_out/bnb_1_h3p.txt
rm -rf $d
