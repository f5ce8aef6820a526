#!/bin/bash
# Round-2 bench matrix on 1 GPU: headline (global pipeline, reference BN
# numerics), folded-BN pipeline, BASELINE config #2 (whole model, one video per
# call) and the fused single-process engine.
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
  tail -n ${TAILN:-4} "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step fb_global_batch 600 python bench.py --steps ${STEPS:-10} --warmup 2 --json-out gpurun_out/fb_global_batch.json
step fb_global_eval 600 python bench.py --bn eval --steps ${STEPS:-10} --warmup 2 --json-out gpurun_out/fb_global_eval.json
step fb_whole_batch 600 python bench.py --pipeline whole --steps 4 --warmup 1 --json-out gpurun_out/fb_whole_batch.json
step fb_fused_eval 600 python bench.py --pipeline fused --steps 10 --warmup 2 --json-out gpurun_out/fb_fused_eval.json
