#!/bin/bash
# x6 (split-bf16 fp32) Winograd kernels: numerics tests, then per-layer
# timing of the fp32 R(2+1)D-34 forward with fp32-MFMA vs x6 Winograd.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py -x -v --timeout 120 --timeout-method thread -k "winograd" > gpurun_out/x6_tests.log 2>&1
rc=$?; tail -n 30 gpurun_out/x6_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/profile_layers.py --depth 34 --clips 128 --dtype fp32 --list-wino --reps 5 > gpurun_out/x6_layers.log 2>&1
rc=$?; grep -E "wino|TOTAL" gpurun_out/x6_layers.log | tail -40; exit $rc
