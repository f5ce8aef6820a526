#!/bin/bash
# Launcher (benchmark.py) runs of the pipeline configs on one MI355X:
# the reference's published setup (r2p1d-whole, 500 videos, -mi 90) for
# R(2+1)D-18 and -34, saturation (-mi 0) runs, and 1-GPU replicate/batch
# topologies. Every run has its own time limit; a crash stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pipelines
export PYTHONUNBUFFERED=1 RNB_NO_TQDM=1
run() {  # run <name> <timeout> <args...>
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" python benchmark.py --log-root gpurun_out/pipelines/logs \
      --json-out "gpurun_out/pipelines/$name.json" --barrier-timeout 300 "$@" \
      > "gpurun_out/pipelines/$name.log" 2>&1
  local rc=$?
  grep -E "Throughput|ERROR|Error" "gpurun_out/pipelines/$name.log" | tail -3
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
python -m rnb_amd.build > /dev/null || exit 3
run whole-r18-mi90 300 -c configs/r2p1d-whole-r18.json -v 500 -mi 90
run whole-r34-mi90 300 -c configs/r2p1d-whole.json -v 500 -mi 90
run whole-r34-mi0 300 -c configs/r2p1d-whole.json -v 2000 -mi 0
run whole-r18-mi0 300 -c configs/r2p1d-whole-r18.json -v 2000 -mi 0
run replicated-1gpu-mi0 400 -c configs/r2p1d-replicated-1gpu.json -v 3000 -mi 0
run rnb-1gpu-mi0 400 -c configs/rnb-1gpu.json -v 3000 -mi 0
run replicated-1gpu-mi2 400 -c configs/r2p1d-replicated-1gpu.json -v 3000 -mi 2
python scripts/parse_logs.py gpurun_out/pipelines/logs --skip 10 > gpurun_out/pipelines/summary.txt 2>&1
cat gpurun_out/pipelines/summary.txt
