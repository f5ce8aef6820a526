#!/bin/bash
# One GPU-box session: build, GPU tests, smoke, short bench. Each GPU step has
# its own time limit; a crash/abort/timeout (rc not in {0,1}) stops the script.
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
step build 600 python -m rnb_amd.build
# TESTS: pytest targets (default: the whole GPU suite); NO_BENCH=1 skips the bench
step pytest_gpu "${PYTEST_TIMEOUT:-900}" python -u -m pytest ${TESTS:-tests} -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
if [ -z "${NO_BENCH:-}" ]; then
  step bench "${BENCH_TIMEOUT:-900}" python bench.py --steps "${BENCH_STEPS:-10}" --warmup 2 --json-out gpurun_out/bench.json ${BENCH_ARGS:-}
fi
