#!/bin/bash
# round 5: literal config #2 (one loader + one runner, one video per call) with
# 2 / 3 / 4 runner lanes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
W="--pipeline whole --replicas 1 --loaders 1 --steps 4 --videos-per-step 128 --latency-mi 10 --latency-load 0 --latency-seconds 3"
timeout -k 10 1100 python scripts/ab_bench.py --rounds 2 --out gpurun_out/ab_lanes_whole.txt \
  "l2||$W --lanes 2" "l3||$W --lanes 3" "l4||$W --lanes 4"
rc=$?; cat gpurun_out/ab_lanes_whole.txt; exit $rc
