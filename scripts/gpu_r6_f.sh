#!/bin/bash
# round 6: first GPU pass of the Winograd h3 kernel (conv_h3w): its numerics
# tests, then the per-layer table of every h3 candidate on the stride-1
# spatial convs (with and without the input BN on load) at 128 clips
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
  tail -n 40 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step h3w_tests 400 python -u -m pytest tests/test_gpu_h3w.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
step h3w_layers 600 python -u scripts/h3_layer_bench.py --clips 128 --only-h3 --cases k3,k3a,k7,k7a,k13,k13a,k19,k19a
