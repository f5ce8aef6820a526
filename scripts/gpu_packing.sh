#!/bin/bash
# A/B of bench.py batch packing on one box: first-fit + 4-clip buckets (default) vs arrival + 8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_ff4.log 2>&1 || exit $?
tail -1 gpurun_out/bench_ff4.log | cut -c1-330
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --packing arrival --bucket-step 8 > gpurun_out/bench_arr8.log 2>&1 || exit $?
tail -1 gpurun_out/bench_arr8.log | cut -c1-330
