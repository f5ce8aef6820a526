#!/bin/bash
# round 6: (1) re-tune from scratch at the new defaults (geo8 buckets) into a
# cache that becomes the seed table; (2) a folded 3-GPU rehearsal of the
# driver's multi-GPU bench at the DEFAULT process counts (2 loaders + 3
# runners per logical GPU = 15 GPU processes on the one card), seeded by (1)
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
  tail -n 12 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
rm -f gpurun_out/tune_cache_r6b.json
RNB_TUNE_SEED=0 RNB_TUNE_CACHE=$PWD/gpurun_out/tune_cache_r6b.json \
  step bench_noseed_geo8 600 python bench.py --json-out gpurun_out/bench_r6_noseed_geo8.json
RNB_TUNE_SEED=$PWD/gpurun_out/tune_cache_r6b.json RNB_FOLD_GPUS=1 \
  RNB_TUNE_CACHE=$PWD/gpurun_out/tune_cache_fold3.json \
  step fold3 900 python bench.py --gpus 3 --json-out gpurun_out/bench_r6_fold3.json
