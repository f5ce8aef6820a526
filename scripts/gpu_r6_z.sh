#!/bin/bash
# round 6: bigger bulk calls (clip / video caps of a model call) vs the
# defaults, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1500 python scripts/ab_bench.py --rounds 2 --steps 10 --timeout 330 \
  --out gpurun_out/ab_callsize.txt \
  "base||" "c320|| --clips-per-batch 320 --video-batch 160" \
  "c384|| --clips-per-batch 384 --video-batch 192"
