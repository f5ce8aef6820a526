#!/bin/bash
# round 5: 16-channel last chunk in the temporal band kernel (Cin_p % 32 == 16:
# conv2 temporal 144, stem temporal 48) -- band tests, layer table, forward
# breakdown at 128 clips, then a traced bench (GPU busy, kernel families)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
trace_of() { ls $1/*/*/run_kernel_trace.csv $1/*/run_kernel_trace.csv $1/run_kernel_trace.csv 2>/dev/null | tail -1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_h3.py -x -q --timeout 120 --timeout-method thread \
  -k "band" > gpurun_out/half_tests.log 2>&1 || { tail -30 gpurun_out/half_tests.log; exit 1; }
tail -3 gpurun_out/half_tests.log
timeout -k 10 300 python scripts/h3_layer_bench.py --clips 128 --cases k4,stemt,stem > gpurun_out/half_layers.txt 2>&1 || { tail gpurun_out/half_layers.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/half_layers.txt | awk '{c[$1]++} c[$1]<=4'
timeout -k 10 240 python scripts/h3t_exp.py --cases k4,stemt > gpurun_out/half_exp.txt 2>&1 || { tail gpurun_out/half_exp.txt; exit 1; }
cat gpurun_out/half_exp.txt
d=gpurun_out/bnb_128; rm -rf $d
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
  -- python3 scripts/bn_breakdown.py run --mode batch --clips 128 > $d.log 2>&1 || { echo "bnb failed"; tail $d.log; exit 1; }
python3 scripts/bn_breakdown.py parse "$(trace_of $d)" --kernels 16 > gpurun_out/bnb_128.txt
head -30 gpurun_out/bnb_128.txt
d=gpurun_out/trb; rm -rf $d
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
  -- python3 bench.py --steps 10 --warmup 2 --no-literal --no-check --json-out gpurun_out/trb.json > gpurun_out/trb.log 2>&1 || { echo "traced bench failed"; tail gpurun_out/trb.log; exit 1; }
python3 scripts/bench_busy.py "$(trace_of $d)" > gpurun_out/trb_busy.txt 2>&1
cat gpurun_out/trb_busy.txt | head -40
rm -rf $d gpurun_out/bnb_128
