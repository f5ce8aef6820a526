#!/bin/bash
# round 6: literal config #2 (3 lanes) tuned from scratch with and without the
# split-K configs (they minimise one call's latency by spreading a small conv
# over many blocks, at extra total work: three calls in flight share the GPU)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out logs/bench
export PYTHONUNBUFFERED=1 RNB_TUNE_SEED=0
base="--gpus 1 --no-literal --no-check --pipeline whole --replicas 1 --loaders 1 --steps 4 --warmup 1 --videos-per-step 128 --latency-seconds 0"
for round in 0 1; do
for v in "ks:" "noks:RNB_X6K=0"; do
  name=${v%%:*}; envs=${v#*:}
  rm -f gpurun_out/tc_$name.json
  env $envs RNB_TUNE_CACHE=$PWD/gpurun_out/tc_$name.json timeout -k 10 400 python bench.py $base --json-out gpurun_out/lit2k_$name.json > gpurun_out/lit2k_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/lit2k_$name.log; exit 1; }
  python3 -c "import json; j=json.load(open('gpurun_out/lit2k_$name.json')); print('$round $name', j['value'], j['ms_per_step'])"
done
done
