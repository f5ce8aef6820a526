#!/bin/bash
# round 6: where a mi = 10 request's latency goes (tail vs median stages)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-literal --no-check --json-out gpurun_out/bench_mi10.json > gpurun_out/bench_mi10.log 2>&1 || exit $?
python3 -c "
import json; j=json.load(open('gpurun_out/bench_mi10.json')); m=j['latency_mi10']; print(json.dumps(m, indent=1))"
