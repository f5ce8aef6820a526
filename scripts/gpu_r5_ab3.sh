#!/bin/bash
# round 5: bulk calls end on an empty queue (~76 rows): do more loaders / replicas help?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1080 python scripts/ab_bench.py --rounds 2 --out gpurun_out/ab_loaders.txt \
  "base||--steps 10" "ld3||--steps 10 --loaders 3" "ld3r4||--steps 10 --loaders 3 --replicas 4"
rc=$?; cat gpurun_out/ab_loaders.txt; exit $rc
