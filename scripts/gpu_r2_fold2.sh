#!/bin/bash
# --gpus 2 rehearsal of the driver's multi-GPU bench on ONE device: torchrun
# with 2 ranks (gloo coordination), RNB_FOLD_GPUS=1 folds logical GPUs 0, 1
# onto the one device (every process / ring / queue as at 2 GPUs). The
# two-stage extra needs 2 physical GPUs (one RCCL rank per GPU) and is
# expected to report an error here.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0 RNB_FOLD_GPUS=1
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 2 --steps ${STEPS:-6} --warmup 1 \
  --cross-gpu-timeout 200 --json-out gpurun_out/fold2.json > gpurun_out/fold2.log 2>&1
rc=$?; grep -E "cross-GPU|Throughput|RNB_FOLD" gpurun_out/fold2.log | tail -n 8; tail -n 2 gpurun_out/fold2.log
exit $rc
