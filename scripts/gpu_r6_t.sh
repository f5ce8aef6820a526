#!/bin/bash
# round 6: BN finalize folded into the producer conv (bn_tail.h) and the
# in-kernel split-K fix-up -- GPU tests, 1 / 4 / 16-clip forward dispatch
# tables, then a bench at the driver defaults
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_bn_tail.py tests/test_gpu_h3.py tests/test_gpu_h3w.py \
  tests/test_gpu_range_guard.py > gpurun_out/t_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_tests.log; exit 1; }
tail -3 gpurun_out/t_tests.log
trace_of() { ls $1/*/*/run_kernel_trace.csv $1/*/run_kernel_trace.csv $1/run_kernel_trace.csv 2>/dev/null | tail -1; }
for c in 1 4 16; do
  d=gpurun_out/bnbt_$c; rm -rf $d
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
    -- python3 scripts/bn_breakdown.py run --mode batch --clips $c > $d.log 2>&1 || { echo "bnb $c failed"; tail $d.log; exit 1; }
  python3 scripts/bn_breakdown.py parse "$(trace_of $d)" --kernels 16 > gpurun_out/bnbt_$c.txt
  head -14 gpurun_out/bnbt_$c.txt
  rm -rf $d
done
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_t.json > gpurun_out/bench_t.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_t.log; exit 1; }
tail -1 gpurun_out/bench_t.log | cut -c1-300
python3 - <<'PY'
import json
j = json.load(open('gpurun_out/bench_t.json'))
print('value', j['value'], 'p50', j['p50_ms'], 'p99', j['p99_ms'], 'mi10', j['latency_mi10'])
print('literal', {k: (v['videos_per_s'], v.get('lanes')) for k, v in j.get('literal', {}).items()})
print('gather bulk', j['gather']['bulk']['rows_per_call'], 'setup', j.get('headline', {}).get('setup'))
PY
