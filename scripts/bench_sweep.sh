#!/bin/bash
# Sweep bench.py knobs on one GPU (each run bounded).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
python -m rnb_amd.build > /dev/null || exit 3
for cfg in ${SWEEP:-"64 2 128" "64 2 96" "64 2 192" "64 3 128" "64 1 256" "32 4 64"}; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps ${STEPS:-6} --warmup 2 --video-batch $1 --replicas $2 --clips-per-batch $3 --videos-per-step ${VPS:-256} > gpurun_out/sweep/vb$1_r$2_c$3.log 2>&1
  rc=$?
  echo "vb=$1 r=$2 c=$3 rc=$rc $(grep -o "\"value\": [0-9.]*" gpurun_out/sweep/vb$1_r$2_c$3.log) $(grep -o "\"p50_ms\": [0-9.]*, \"p99_ms\": [0-9.]*" gpurun_out/sweep/vb$1_r$2_c$3.log)"
  [ $rc -le 1 ] || exit $rc
done
