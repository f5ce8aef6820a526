#!/bin/bash
# round 5: the pixel-major temporal kernel in the whole pipeline
# (RNB_H3P 0 / 1, each with its own tuning cache), 10 steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1150 python scripts/ab_bench.py --rounds 3 --timeout 240 --out gpurun_out/ab_h3p_pipeline.txt \
  "h3p0|RNB_H3P=0,RNB_TUNE_CACHE=/tmp/tc_h3p0.json|--steps 10" "h3p1|RNB_H3P=1,RNB_TUNE_CACHE=/tmp/tc_h3p1.json|--steps 10"
rc=$?; cat gpurun_out/ab_h3p_pipeline.txt; exit $rc
