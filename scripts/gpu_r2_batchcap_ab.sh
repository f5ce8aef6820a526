#!/bin/bash
# Headline model-call capacity A/B (3 runner replicas): 64 videos / 128 clips
# (default) vs 96 videos / 192 clips per call, interleaved, 20 steps each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 RNB_TUNE_CACHE=$PWD/gpurun_out/tune_cap.json
i=0
for cap in ${CAPS:-128:64 192:96 128:64 192:96}; do
  c=${cap%%:*}; v=${cap##*:}; i=$((i+1))
  log=gpurun_out/cap_${i}_c${c}_v${v}
  timeout -k 10 500 python bench.py --clips-per-batch $c --video-batch $v --steps ${STEPS:-20} \
    --warmup 2 --json-out $log.json > $log.log 2>&1
  rc=$?; echo "=== $i: clips $c videos $v rc=$rc"; grep -E "Throughput|Latency phase" $log.log
  [ $rc -eq 0 ] || exit $rc
done
