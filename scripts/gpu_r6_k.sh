#!/bin/bash
# round 6: full GPU suite + smoke on the current tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r6.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu_r6.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6.log 2>&1
rc2=$?; tail -3 gpurun_out/smoke_r6.log; exit $(( rc > rc2 ? rc : rc2 ))
