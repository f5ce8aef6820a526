#!/bin/bash
# round 6: (1) re-tune from scratch with the h3w configs in the autotune set
# (geo8 buckets) into a cache that becomes the seed table; (2) a folded 2-GPU
# rehearsal of the driver's multi-GPU bench at the DEFAULT process counts (2
# loaders + 3 runners per logical GPU = 10 GPU processes on the one card;
# 3 logical GPUs = 15 processes ran the card out of memory, fold3.log), seeded by (1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 6 "gpurun_out/$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step h3w_tests 300 python -u -m pytest tests/test_gpu_h3w.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
rm -f gpurun_out/tune_cache_r6j.json
RNB_TUNE_SEED=0 RNB_TUNE_CACHE=$PWD/gpurun_out/tune_cache_r6j.json \
  step bench_noseed_h3w 600 python bench.py --json-out gpurun_out/bench_r6_noseed_h3w.json
RNB_TUNE_SEED=$PWD/gpurun_out/tune_cache_r6j.json RNB_FOLD_GPUS=1 \
  RNB_TUNE_CACHE=$PWD/gpurun_out/tune_cache_fold2.json \
  step fold2 900 python bench.py --gpus 2 --json-out gpurun_out/bench_r6_fold2.json
