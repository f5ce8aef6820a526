#!/bin/bash
# BASELINE config #2 shape (whole model, one video per model call, batch BN):
# runner replicas per GPU 2 / 3 / 4 with 2 loaders.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 RNB_TUNE_CACHE=$PWD/gpurun_out/tune_whole.json
for r in ${REPLICAS:-2 3 4}; do
  timeout -k 10 400 python bench.py --pipeline whole --replicas $r --loaders 2 --steps 4 --warmup 1 \
    --json-out gpurun_out/whole_r$r.json > gpurun_out/whole_r$r.log 2>&1
  rc=$?; echo "=== replicas $r rc=$rc"; grep -E "Throughput|Latency phase" gpurun_out/whole_r$r.log
  [ $rc -eq 0 ] || exit $rc
done
