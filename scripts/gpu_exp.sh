#!/bin/bash
# Kernel tests + per-layer table + bottleneck experiment for selected layers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider > gpurun_out/kt.log 2>&1
rc=$?; tail -3 gpurun_out/kt.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python scripts/profile_layers.py --depth 34 --clips 64 --autotune --json-out gpurun_out/layers2.json > gpurun_out/layers2.log 2>&1
rc=$?; tail -1 gpurun_out/layers2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/kernel_exp.py run --configs "${EXP_CONFIGS:-}" --layers "${EXP_LAYERS:-conv2.blocks.0.conv1.spatial,conv2.blocks.0.conv1.temporal,conv2.blocks.0.conv2.temporal,conv3.blocks.0.conv1.spatial,conv3.blocks.0.conv2.temporal}" > gpurun_out/exp.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/exp.log; exit $rc
