#!/bin/bash
# Kernel iteration: tests, per-layer table, then counters for one conv.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
HEADN=${HEADN:-20} bash scripts/gpu_kernels.sh || exit $?
bash scripts/gpu_pmc.sh || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc
