#!/bin/bash
# round 6 final tree: the driver's exact N>1 launch form (torchrun, one rank
# per logical GPU) folded onto the one card at the default process counts
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
RNB_FOLD_GPUS=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --json-out gpurun_out/bench_r6_torchrun_fold2_final.json \
  > gpurun_out/torchrun_fold2_final.log 2>&1
rc=$?; tail -2 gpurun_out/torchrun_fold2_final.log | cut -c1-600; exit $rc
