#!/bin/bash
# round 6 final tree: graphed forward dispatch / family tables at 1, 4, 16 and
# 128 clips
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
trace_of() { ls $1/*/*/run_kernel_trace.csv $1/*/run_kernel_trace.csv $1/run_kernel_trace.csv 2>/dev/null | tail -1; }
for c in 1 4 16 128; do
  d=gpurun_out/bnbf_$c; rm -rf $d
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
    -- python3 scripts/bn_breakdown.py run --mode batch --clips $c > $d.log 2>&1 || { echo "bnb $c failed"; tail $d.log; exit 1; }
  python3 scripts/bn_breakdown.py parse "$(trace_of $d)" --kernels 24 > gpurun_out/bnbf_$c.txt
  head -3 gpurun_out/bnbf_$c.txt
  rm -rf $d
done
