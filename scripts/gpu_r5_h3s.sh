#!/bin/bash
# round 5: stride-2 row-band h3 kernel (conv_h3s) -- its tests, the stride-2
# layer table, and the 128-clip forward breakdown with h3s in the autotune set
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
trace_of() { ls $1/*/*/run_kernel_trace.csv $1/*/run_kernel_trace.csv $1/run_kernel_trace.csv 2>/dev/null | tail -1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_h3.py tests/test_gpu_f32.py -x -q --timeout 120 --timeout-method thread \
  -k "h3s or walk_apply" > gpurun_out/h3s_tests.log 2>&1 || { tail -40 gpurun_out/h3s_tests.log; exit 1; }
tail -3 gpurun_out/h3s_tests.log
RNB_H3S=1 timeout -k 10 300 python scripts/h3_layer_bench.py --clips 128 --cases k5,k11,k17 --only-h3 > gpurun_out/h3s_layers.txt 2>&1 || { tail gpurun_out/h3s_layers.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/h3s_layers.txt | awk '{c[$1]++} c[$1]<=6'
d=gpurun_out/bnb_128; rm -rf $d
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
  -- python3 scripts/bn_breakdown.py run --mode batch --clips 128 > $d.log 2>&1 || { echo "bnb failed"; tail $d.log; exit 1; }
python3 scripts/bn_breakdown.py parse "$(trace_of $d)" --kernels 18 > gpurun_out/bnb_128.txt
head -34 gpurun_out/bnb_128.txt
rm -rf $d
