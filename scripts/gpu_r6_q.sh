#!/bin/bash
# round 6: the range-guard tests (uses_h3), then the driver's exact N>1 launch
# form (torchrun, one rank per logical GPU) folded onto the one card at the
# default process counts (2 logical GPUs = 10 GPU processes)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_range_guard.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/guard_tests.log 2>&1
rc=$?; tail -3 gpurun_out/guard_tests.log; [ $rc -eq 0 ] || exit $rc
RNB_FOLD_GPUS=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --json-out gpurun_out/bench_r6_torchrun_fold2.json \
  > gpurun_out/torchrun_fold2.log 2>&1
rc=$?; tail -3 gpurun_out/torchrun_fold2.log | cut -c1-400; exit $rc
