#!/bin/bash
# Sweep bench.py batching / replication knobs (default 1-GPU config otherwise).
#   bash scripts/bench_sweep.sh ["VIDEO_BATCH CLIPS_PER_BATCH REPLICAS" ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
python -m rnb_amd.build > /dev/null || exit 3
[ $# -gt 0 ] || set -- "64 128 3" "64 192 3" "64 256 2" "64 96 4" "64 128 4" "96 192 2"
for cfg in "$@"; do
  set -- $cfg
  name="vb$1_c$2_r$3"
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --video-batch $1 \
      --clips-per-batch $2 --replicas $3 > gpurun_out/sweep/$name.log 2>&1
  rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*, ' gpurun_out/sweep/$name.log) \
$(grep -o '"p50_ms": [0-9.]*, "p99_ms": [0-9.]*' gpurun_out/sweep/$name.log)"
  [ $rc -eq 0 ] || exit $rc
done
