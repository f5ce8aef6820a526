#!/bin/bash
# round 5: where did the headline go (1580 -> ~1390)? lane stream priority and the h3 range guard
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1080 python scripts/ab_bench.py --rounds 2 --out gpurun_out/ab_prio_guard.txt \
  "base||--steps 10" "lane0|RNB_LANE_PRIORITY=0|--steps 10" "noguard|RNB_H3_GUARD=0|--steps 10" \
  "both|RNB_LANE_PRIORITY=0,RNB_H3_GUARD=0|--steps 10"
rc=$?; cat gpurun_out/ab_prio_guard.txt; exit $rc
