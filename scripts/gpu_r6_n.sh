#!/bin/bash
# round 6: what bounds literal config #2 (1 loader + 1 runner, one video per
# call, 3 lanes)? the same run with 2 loaders, and with 6 lanes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out logs/bench
export PYTHONUNBUFFERED=1
base="--gpus 1 --no-literal --no-check --pipeline whole --replicas 1 --steps 4 --warmup 1 --videos-per-step 128 --latency-seconds 0"
for v in "l1:--loaders 1" "l2:--loaders 2" "l1x6:--loaders 1 --lanes 6" "l1x1:--loaders 1 --lanes 1" "l3:--loaders 3"; do
  name=${v%%:*}; extra=${v#*:}
  timeout -k 10 300 python bench.py $base $extra --json-out gpurun_out/lit2_$name.json > gpurun_out/lit2_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/lit2_$name.log; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/lit2_$name.json')); print('$name', j['value'], j['ms_per_step'], j['config']['parallelism'], j['config'].get('lanes'))"
done
