#!/bin/bash
# round 6: work-conserving overflow of 15-clip videos to the 1-clip-video
# replicas (--large-overflow k) -- bulk throughput and the Poisson tails,
# interleaved rounds against the default routing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1500 python scripts/ab_bench.py --rounds 2 --steps 10 --timeout 300 \
  --out gpurun_out/ab_overflow.txt \
  "base||--latency-seconds 6" "ovf1||--latency-seconds 6 --large-overflow 1" \
  "ovf3||--latency-seconds 6 --large-overflow 3"
