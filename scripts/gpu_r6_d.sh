#!/bin/bash
# round 6: the new wide h3 direct configs (13-17): numerics tests, then the
# per-layer table of every h3 candidate on the GEMM-shaped convs at 128 clips,
# then the CU-mask Poisson-tail A/B
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
step h3tests 600 python -u -m pytest tests/test_gpu_h3.py tests/test_gpu_cumask.py -q -p no:cacheprovider --timeout 120 --timeout-method thread
step layers 900 python -u scripts/h3_layer_bench.py --clips 128 --only-h3 --cases k8,k14,k20,k19,k12,k18,k5,k11,k17,k6
bash scripts/gpu_r6_c.sh
