#!/bin/bash
# Headline pipeline (aggressive = global at 1 GPU, batch BN): loader / runner
# process counts per GPU, 10 steps each, one shared tile cache.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 RNB_TUNE_CACHE=$PWD/gpurun_out/tune_head.json
for lr in ${LR:-2:2 2:3 3:3 2:2}; do
  l=${lr%%:*}; r=${lr##*:}
  timeout -k 10 400 python bench.py --loaders $l --replicas $r --steps 10 --warmup 2 \
    --json-out gpurun_out/head_l${l}_r${r}.json > gpurun_out/head_l${l}_r${r}.log 2>&1
  rc=$?; echo "=== loaders $l replicas $r rc=$rc"; grep -E "Throughput|Latency phase" gpurun_out/head_l${l}_r${r}.log
  [ $rc -eq 0 ] || exit $rc
done
