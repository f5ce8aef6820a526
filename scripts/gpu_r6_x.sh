#!/bin/bash
# round 6: full GPU suite + smoke + a bench at the driver defaults on the
# current tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r6x.log 2>&1
rc=$?
tail -8 gpurun_out/pytest_gpu_r6x.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r6x.log 2>&1 || { tail gpurun_out/smoke_r6x.log; exit 1; }
tail -2 gpurun_out/smoke_r6x.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 560 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_r6x.json > gpurun_out/bench_r6x.log 2>&1 || { tail -20 gpurun_out/bench_r6x.log; exit 1; }
python3 - <<'PY'
import json
j = json.load(open('gpurun_out/bench_r6x.json'))
print('value', j['value'], 'p50', j['p50_ms'], 'p99', j['p99_ms'], 'mi10', {k: j['latency_mi10'][k] for k in ('p50_ms', 'p99_ms')})
print('literal', {k: (v['videos_per_s'], v.get('lanes')) for k, v in j.get('literal', {}).items()})
print('gather bulk', j['gather']['bulk']['rows_per_call'], 'tuned', j['model_counters'].get('tune_tuned'), 'numerics', j['numerics']['max_rel_err'], j['numerics']['top1_agree'])
PY
