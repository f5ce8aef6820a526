#!/bin/bash
# Sweep bench.py knobs on one GPU (each run bounded).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
python -m rnb_amd.build > /dev/null || exit 3
for cfg in ${SWEEP:-"32 1" "32 2" "64 1" "64 2" "16 4" "128 1"}; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps ${STEPS:-6} --warmup 2 --video-batch $1 --replicas $2 --videos-per-step $(( $1 * ${MULT:-4} )) > gpurun_out/sweep/vb$1_r$2.log 2>&1
  rc=$?
  echo "vb=$1 r=$2 rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/sweep/vb$1_r$2.log) $(grep -o '"p50_ms": [0-9.]*, "p99_ms": [0-9.]*' gpurun_out/sweep/vb$1_r$2.log)"
  [ $rc -le 1 ] || exit $rc
done
