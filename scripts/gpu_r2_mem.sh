#!/bin/bash
# Runner memory after largest-first bucket capture: default bench (128 clips)
# and 192-clip model calls, 3 runner replicas, memory reported per runner.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 RNB_REPORT_MEMORY=1 RNB_TUNE_CACHE=$PWD/gpurun_out/tune_mem.json
i=0
for cap in ${CAPS:-128:64 192:96 128:64 192:96}; do
  c=${cap%%:*}; v=${cap##*:}; i=$((i+1))
  log=gpurun_out/mem_${i}_c${c}_v${v}
  timeout -k 10 500 python bench.py --clips-per-batch $c --video-batch $v --steps 20 --warmup 2 \
    --json-out $log.json > $log.log 2>&1
  rc=$?; echo "=== $i: clips $c videos $v rc=$rc"; grep -E "GB reserved|Throughput|Latency phase" $log.log
  [ $rc -eq 0 ] || exit $rc
done
