#!/bin/bash
# bn_breakdown of one graphed batch-BN forward under two environments (A/B):
#   bash scripts/bnbreak_ab.sh CLIPS "ENV_A" "ENV_B"   (e.g. "RNB_BN_FUSED_FINALIZE=32")
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
c=$1; shift
i=0
for envs in "$@"; do
  i=$((i+1)); d=gpurun_out/bnbab_${c}_$i
  rm -rf $d
  env $envs timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
    -- python3 scripts/bn_breakdown.py run --mode batch --clips "$c" > $d.log 2>&1 || { echo "run $i failed"; exit 1; }
  trace=$(ls $d/*/*/run_kernel_trace.csv $d/*/run_kernel_trace.csv $d/run_kernel_trace.csv 2>/dev/null | tail -1)
  echo "== $envs"
  python3 scripts/bn_breakdown.py parse "$trace" --kernels 8 | head -16
done
