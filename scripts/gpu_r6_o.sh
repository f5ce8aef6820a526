#!/bin/bash
# round 6: host-time profile of the literal config #2 runner and loader
# (RNB_PROFILE_STAGES=1), 3 lanes and 1 lane
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out logs/bench
export PYTHONUNBUFFERED=1 RNB_PROFILE_STAGES=1
base="--gpus 1 --no-literal --no-check --pipeline whole --replicas 1 --loaders 1 --steps 4 --warmup 1 --videos-per-step 128 --latency-seconds 0"
for v in "x3:--lanes 3" "x1:--lanes 1"; do
  name=${v%%:*}; extra=${v#*:}
  timeout -k 10 300 python bench.py $base $extra --json-out gpurun_out/lit2p_$name.json > gpurun_out/lit2p_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/lit2p_$name.log; exit 1; }
  echo "== $name"; grep -iE "host time|stages|profile" gpurun_out/lit2p_$name.log | head -10
done
