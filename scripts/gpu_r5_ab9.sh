#!/bin/bash
# round 5: latency-regime lane priority for the 15-clip-video replica
# (RNB_LATENCY_PRIORITY 0 = default-priority lanes always, 1 = the group's
# priority while few requests are queued), 10 steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1150 python scripts/ab_bench.py --rounds 3 --timeout 200 --out gpurun_out/ab_latency_priority.txt \
  "prio0|RNB_LATENCY_PRIORITY=0|--steps 10" "prio1|RNB_LATENCY_PRIORITY=1|--steps 10"
rc=$?; cat gpurun_out/ab_latency_priority.txt; exit $rc
