#!/bin/bash
# Host-phase profile of the pipeline bench (event vs host slot ordering).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 RNB_PROFILE_STAGES=1
for order in ${ORDERS:-event host}; do
  name="prof_${order}${TAG:-}"
  echo "=== $name"
  RNB_RING_ORDER=$order timeout -k 10 600 python bench.py --loaders ${L:-2} --replicas ${R:-2} --steps 10 --warmup 2 --latency-seconds 0 ${EXTRA:-} > gpurun_out/$name.log 2>&1
  rc=$?
  echo "=== $name rc=$rc"
  grep -E "host time|batched calls|Throughput" gpurun_out/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
