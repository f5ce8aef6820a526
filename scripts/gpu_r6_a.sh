#!/bin/bash
# round 6, first GPU pass: GPU suite, smoke, then a bench at the driver's
# defaults that tunes from scratch (no seed table) into its own cache file --
# the tune-cache fix shows as tuned > 0 for one replica only -- and that file
# becomes the seed table (rnb_amd/ops/tune_seed.json)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
rm -f gpurun_out/tune_cache_r6.json
RNB_TUNE_SEED=0 RNB_TUNE_CACHE=$PWD/gpurun_out/tune_cache_r6.json \
  step bench_noseed 600 python bench.py --json-out gpurun_out/bench_r6_noseed.json
