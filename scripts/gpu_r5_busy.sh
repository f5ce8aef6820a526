#!/bin/bash
# round 5: where the bulk phase loses GPU time -- traced bench (all processes'
# kernel traces merged: busy per 0.5-s window, per dispatching thread, idle
# gaps), and the stem convs' candidates
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python scripts/h3_layer_bench.py --clips 128 --cases stem,stemt > gpurun_out/stem_layers.txt 2>&1 || { tail gpurun_out/stem_layers.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stem_layers.txt | awk '{c[$1]++} c[$1]<=6'
d=gpurun_out/trb; rm -rf $d
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
  -- python3 bench.py --steps 30 --warmup 2 --no-literal --no-check --json-out gpurun_out/trb.json > gpurun_out/trb.log 2>&1 || { echo "traced bench failed"; tail gpurun_out/trb.log; exit 1; }
timeout -k 10 300 python3 scripts/bench_busy.py $d > gpurun_out/trb_busy.txt 2>&1
cat gpurun_out/trb_busy.txt | head -60
grep -E "bulk:|latency:" gpurun_out/trb.log | head
rm -rf $d
