#!/bin/bash
# round 6: the Winograd h3 kernel at small call sizes (1 / 4 / 16 clips),
# every candidate of the stride-1 spatial convs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for n in 1 4 16; do
  timeout -k 10 400 python -u scripts/h3_layer_bench.py --clips $n --cases k3,k3a,k7,k7a,k13,k13a,k19,k19a \
    > gpurun_out/h3w_small_$n.log 2>&1 || exit $?
  echo "== clips $n"; for c in k3 k3a k7 k7a k13 k13a k19 k19a; do grep -E "^$c " gpurun_out/h3w_small_$n.log | head -3; grep -E "^$c .*cid 146[01]" gpurun_out/h3w_small_$n.log; done
done
