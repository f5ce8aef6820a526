#!/bin/bash
# Profiling session: per-layer table + rocprofv3 kernel stats of bench.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-60} "gpurun_out/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
python -m rnb_amd.build > /dev/null
run layers 300 python scripts/profile_layers.py --depth 34 --clips ${CLIPS:-64} --autotune --json-out gpurun_out/layers.json
rm -rf gpurun_out/prof
TAILN=5 run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 1
find gpurun_out/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -25 {}'
