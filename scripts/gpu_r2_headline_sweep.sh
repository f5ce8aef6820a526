#!/bin/bash
# Headline pipeline (aggressive = global at 1 GPU, batch BN): loader / runner
# process counts per GPU, 10 steps each, one shared tile cache.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 RNB_TUNE_CACHE=$PWD/gpurun_out/tune_head.json
i=0
for lr in ${LR:-2:2 2:3 3:3 2:2}; do
  l=${lr%%:*}; r=${lr##*:}; i=$((i+1))
  log=gpurun_out/head_${i}_l${l}_r${r}
  timeout -k 10 400 python bench.py --loaders $l --replicas $r --steps ${STEPS:-10} --warmup 2 \
    --json-out $log.json > $log.log 2>&1
  rc=$?; echo "=== $i: loaders $l replicas $r rc=$rc"; grep -E "Throughput|Latency phase" $log.log
  [ $rc -eq 0 ] || exit $rc
done
