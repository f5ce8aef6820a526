#!/bin/bash
# round 5: whole GPU suite (with the IPC soak's printout), smoke, then the
# per-dispatch MFMA / clock counters of one 128-clip forward
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1
rc=$?; grep -E "ipc-soak|ipc-rotate|ipc-scale|passed|failed|FAIL|ERROR" gpurun_out/pytest_gpu_full.log | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 1; }
d=gpurun_out/pmcf; rm -rf $d
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES \
  --kernel-trace --output-format csv -d $d -o run -- python3 scripts/bn_breakdown.py run --mode batch --clips 128 --reps 1 > $d.log 2>&1 || { tail $d.log; exit 1; }
python3 scripts/pmc_forward.py $d > gpurun_out/pmc_forward_128.txt 2>&1
tail -25 gpurun_out/pmc_forward_128.txt
rm -rf $d
exit $rc
