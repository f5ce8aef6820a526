#!/bin/bash
# Kernel session: numerics tests of every tile config, then the per-layer table.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python -m rnb_amd.build > /dev/null || exit 3
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider > gpurun_out/kt.log 2>&1
rc=$?
tail -5 gpurun_out/kt.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python scripts/profile_layers.py --depth 34 --clips ${CLIPS:-64} --autotune ${COMPARE:+--compare} --json-out gpurun_out/layers2.json > gpurun_out/layers2.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/layers2.log | head -${HEADN:-16}
tail -1 gpurun_out/layers2.log
exit $rc
