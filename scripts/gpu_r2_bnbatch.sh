#!/bin/bash
# bn_mode='batch' (reference training-mode BN, per-video statistics): GPU
# tests of the graphed path, then the headline pipeline bench in batch mode.
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
  tail -n ${TAILN:-25} "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step bn_tests 600 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_engine.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "batch_bn or per_video"
TAILN=12 step bench_bnbatch 900 python bench.py --bn batch --steps ${STEPS:-10} --warmup 2 --json-out gpurun_out/bench_bnbatch.json
