#!/bin/bash
# round 5: where the GPU time goes -- traced bench (busy %, families), graphed
# forward breakdowns at 128 and 1 clip, spatial-conv layer table
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
trace_of() { ls $1/*/*/run_kernel_trace.csv $1/*/run_kernel_trace.csv $1/run_kernel_trace.csv 2>/dev/null | tail -1; }
for c in 128 1; do
  d=gpurun_out/bnb_$c; rm -rf $d
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
    -- python3 scripts/bn_breakdown.py run --mode batch --clips $c > $d.log 2>&1 || { echo "bnb $c failed"; tail $d.log; exit 1; }
  python3 scripts/bn_breakdown.py parse "$(trace_of $d)" --kernels 14 > gpurun_out/bnb_$c.txt
  head -30 gpurun_out/bnb_$c.txt
done
timeout -k 10 300 python scripts/h3_layer_bench.py --clips 128 --cases k3,k7,k13,k5,k11 --only-h3 > gpurun_out/layers_spatial.txt 2>&1 || exit 1
grep -B0 -A2 "" gpurun_out/layers_spatial.txt | awk '{print}' | head -80
d=gpurun_out/trb; rm -rf $d
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-literal --no-check --json-out gpurun_out/trb.json > gpurun_out/trb.log 2>&1 || { echo "traced bench failed"; tail gpurun_out/trb.log; exit 1; }
python3 scripts/bench_busy.py "$(trace_of $d)" > gpurun_out/trb_busy.txt 2>&1
cat gpurun_out/trb_busy.txt | head -40
rm -rf $d gpurun_out/bnb_128 gpurun_out/bnb_1
