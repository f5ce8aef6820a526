#!/bin/bash
# round 6: where the GPU time goes with the round-6 seed table (h3w picks for
# small calls): graphed forward breakdowns at 128 / 16 / 1 clips, then a
# traced bench (busy %, families) with rocprofv3 kernel statistics
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
trace_of() { ls $1/*/*/run_kernel_trace.csv $1/*/run_kernel_trace.csv $1/run_kernel_trace.csv 2>/dev/null | tail -1; }
stats_of() { ls $1/*/*/run_kernel_stats.csv $1/*/run_kernel_stats.csv $1/run_kernel_stats.csv 2>/dev/null | tail -1; }
for c in 128 16 1; do
  d=gpurun_out/bnb6_$c; rm -rf $d
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
    -- python3 scripts/bn_breakdown.py run --mode batch --clips $c > $d.log 2>&1 || { echo "bnb $c failed"; tail $d.log; exit 1; }
  python3 scripts/bn_breakdown.py parse "$(trace_of $d)" --kernels 16 > gpurun_out/bnb6_$c.txt
  head -24 gpurun_out/bnb6_$c.txt
done
d=gpurun_out/trb6; rm -rf $d
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-literal --no-check --json-out gpurun_out/trb6.json > gpurun_out/trb6.log 2>&1 || { echo "traced bench failed"; tail gpurun_out/trb6.log; exit 1; }
python3 scripts/bench_busy.py "$(trace_of $d)" > gpurun_out/trb6_busy.txt 2>&1
head -40 gpurun_out/trb6_busy.txt
s="$(stats_of $d)"; [ -n "$s" ] && head -40 "$s" > gpurun_out/trb6_kernel_stats_top.csv
rm -rf $d gpurun_out/bnb6_128 gpurun_out/bnb6_16 gpurun_out/bnb6_1
