#!/bin/bash
# Pipeline bench sweep (fp32, 1 GPU): loaders x replicas.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in ${VARIANTS:-1_2 2_2 3_2 2_3}; do
  set -- ${v//_/ }
  name="sweep_l$1_r$2${TAG:-}"
  echo "=== $name ($(date +%T))"
  timeout -k 10 600 python bench.py --loaders $1 --replicas $2 --steps 10 --warmup 2 ${EXTRA:-} > gpurun_out/$name.log 2>&1
  rc=$?
  echo "=== $name rc=$rc"
  grep -E "batched calls|Throughput|Latency phase" gpurun_out/$name.log
  tail -n 1 gpurun_out/$name.log | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
