#!/bin/bash
# Kernel-family breakdown of the graphed fp32 forward, batch vs eval BN, at
# a full (128) and a typical pipeline (24) clip bucket.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd_root=$(pwd)
for cfg in ${CFGS:-batch:128 eval:128 batch:24 eval:24}; do
  mode=${cfg%%:*}; clips=${cfg##*:}
  name="bnb_${mode}_${clips}"
  echo "=== $name ($(date +%T))"
  rm -rf "gpurun_out/$name"
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "gpurun_out/$name" -o run -- \
    python3 scripts/bn_breakdown.py run --mode "$mode" --clips "$clips" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"
  grep -E "graphed forward|Error|error" "gpurun_out/$name.log" | tail -5
  if [ $rc -ne 0 ]; then exit $rc; fi
  trace=$(ls gpurun_out/$name/*/*/run_kernel_trace.csv gpurun_out/$name/*/run_kernel_trace.csv gpurun_out/$name/run_kernel_trace.csv 2>/dev/null | tail -1)
  python3 scripts/bn_breakdown.py parse "$trace" --kernels ${KERNELS:-12} | tee "gpurun_out/$name.txt"
  rm -f "$trace"
done
