#!/bin/bash
# round 6: fixed (ramp / drain) time of the bulk phase -- bench at 10 / 20 /
# 40 steps (T(K) = a + b K), and the per-replica call timeline of a 20-step run
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for k in 20 10 40; do
  timeout -k 10 400 python bench.py --steps $k --warmup 5 --no-literal --no-check --latency-seconds 0 \
    --latency-mi 0 --json-out gpurun_out/bt_$k.json > gpurun_out/bt_$k.log 2>&1 || { echo "bench $k failed"; tail gpurun_out/bt_$k.log; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/bt_$k.json')); print($k, 'steps', j['value'], 'videos/s', j['ms_per_step'], 'ms/step')"
  if [ $k = 20 ]; then
    d=$(ls -td logs/*/ | grep -v 'logs/bench/' | head -1)
    python3 scripts/bulk_timeline.py "$d" --bin-ms 50 > gpurun_out/bt_timeline_20.txt 2>&1
    head -12 gpurun_out/bt_timeline_20.txt
  fi
done
