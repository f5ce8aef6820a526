#!/bin/bash
# deferred batch-BN (temporal Winograd applies its input BN) + IPC event-wait
# fallback: GPU tests, then the whole-model pipeline and the batch-BN headline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n ${TAILN:-6} "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step defer_tests 600 python -u -m pytest tests/test_gpu_f32.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
step defer_timing 300 python scripts/bn_profile.py
step whole_batch 600 python bench.py --pipeline whole --steps 4 --warmup 1 --json-out gpurun_out/whole_batch.json
step global_batch 600 python bench.py --steps 10 --warmup 2 --json-out gpurun_out/global_batch.json
