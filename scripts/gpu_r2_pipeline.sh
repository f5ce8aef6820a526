#!/bin/bash
# Round-2 pipeline session: GPU pipeline tests, bench.py through the RnB
# launcher (fp32 headline), and the fused engine for comparison.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n ${TAILN:-25} "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pipe_tests 600 python -u -m pytest tests/test_gpu_pipeline.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
TAILN=40 step bench_global 900 python bench.py --steps ${STEPS:-10} --warmup 2 --json-out gpurun_out/bench_global.json
step bench_fused_f32 600 python bench.py --pipeline fused --dtype fp32 --steps 10 --warmup 2 --json-out gpurun_out/bench_fused_f32.json
