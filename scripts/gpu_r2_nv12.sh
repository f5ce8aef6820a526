#!/bin/bash
# NV12 decoder kernels + benches with the NV12 loader.
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
  tail -n ${TAILN:-6} "gpurun_out/$name.log" | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step video_tests 300 python -u -m pytest tests/test_gpu_video.py tests/test_gpu_f32.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
RNB_PROFILE_STAGES=1 TAILN=12 step bench_nv12 900 python bench.py --steps 10 --warmup 2 --json-out gpurun_out/bench_nv12.json
step bench_fused_nv12 600 python bench.py --pipeline fused --dtype fp32 --steps 10 --warmup 2
