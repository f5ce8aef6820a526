#!/bin/bash
# Per-dispatch MFMA counters of one graphed R(2+1)D-34 fp32 forward (batch BN,
# 128 clips): a plain run first fills the tile cache, then ONE counter pass
# (4 counters, --kernel-trace only) replays the graph once after the marker.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1 RNB_TUNE_CACHE=$PWD/gpurun_out/tune_pmcf.json
timeout -k 10 300 python3 scripts/bn_breakdown.py run --mode ${MODE:-batch} --clips 128 --reps 2 \
  > gpurun_out/pmcf_warm.log 2>&1
rc=$?; tail -n 1 gpurun_out/pmcf_warm.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/pmcf
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES \
  --kernel-trace --output-format csv -d gpurun_out/pmcf -o run -- \
  python3 scripts/bn_breakdown.py run --mode ${MODE:-batch} --clips 128 --reps 1 > gpurun_out/pmcf.log 2>&1
rc=$?; tail -n 1 gpurun_out/pmcf.log; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_forward.py gpurun_out/pmcf > gpurun_out/pmc_forward_${MODE:-batch}_128.txt
rc=$?; tail -n 12 gpurun_out/pmc_forward_${MODE:-batch}_128.txt
rm -rf gpurun_out/pmcf
exit $rc
