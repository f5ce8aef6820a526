#!/bin/bash
# fp32 path check: fp32 GPU tests + per-layer fp32 timing.
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
  tail -n ${TAILN:-30} "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step f32_tests 600 python -u -m pytest tests/test_gpu_f32.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
TAILN=80 step f32_layers 600 python scripts/profile_layers.py --depth 34 --clips ${CLIPS:-128} --autotune --dtype fp32 ${PROFILE_ARGS:-}
