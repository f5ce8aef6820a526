#!/bin/bash
# Stem pair-pack check: per-layer table with and without it, bench at driver defaults
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python scripts/profile_layers.py --depth 34 --clips 128 --autotune --fuse > gpurun_out/layers128_stem.txt 2>&1 || exit $?
grep -E "conv1\.|TOTAL" gpurun_out/layers128_stem.txt
RNB_STEM_PACK=0 timeout -k 10 300 python scripts/profile_layers.py --depth 34 --clips 128 --autotune --fuse > gpurun_out/layers128_nostem.txt 2>&1 || exit $?
grep -E "conv1\.|TOTAL" gpurun_out/layers128_nostem.txt
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench20.log 2>&1 || exit $?
tail -1 gpurun_out/bench20.log
