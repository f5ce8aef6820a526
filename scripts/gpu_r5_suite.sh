#!/bin/bash
# round 5 (final): whole GPU suite, then smoke()
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1
rc=$?; grep -E "ipc-soak|passed|failed|FAIL|ERROR" gpurun_out/pytest_gpu_full.log | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
exit $rc
