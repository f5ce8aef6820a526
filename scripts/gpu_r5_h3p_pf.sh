#!/bin/bash
# (historical: the RNB_H3P_PF switch was removed after this A/B, profiles/r5_h3p_touch_prefetch_ab.txt)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_h3.py -x -q --timeout 120 --timeout-method thread \
  -k "h3p or temporal_band" > gpurun_out/h3ppf_tests.log 2>&1 || { tail -40 gpurun_out/h3ppf_tests.log; exit 1; }
tail -2 gpurun_out/h3ppf_tests.log
for pf in 0 1 0 1; do
  RNB_H3P_PF=$pf timeout -k 10 200 python scripts/h3_layer_bench.py --clips 128 --cases k4,stemt --cids 1440 --rounds 3 > gpurun_out/h3ppf_$pf.txt 2>&1 || { tail gpurun_out/h3ppf_$pf.txt; exit 1; }
  echo "PF=$pf"; grep -v amdgpu.ids gpurun_out/h3ppf_$pf.txt
done
