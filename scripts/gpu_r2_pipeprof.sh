#!/bin/bash
# Per-process GPU kernel time of the 1-GPU pipeline bench (loaders vs runners).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
rm -rf gpurun_out/pipeprof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pipeprof -o run -- \
  python3 bench.py --steps ${STEPS:-10} --warmup 2 --latency-seconds 0 ${EXTRA:-} > gpurun_out/pipeprof.log 2>&1
rc=$?
echo "rc=$rc"; grep -E "batched calls|Throughput" gpurun_out/pipeprof.log
[ $rc -ne 0 ] && exit $rc
for f in $(ls gpurun_out/pipeprof/*/*/run_kernel_stats.csv gpurun_out/pipeprof/*/run_kernel_stats.csv 2>/dev/null); do
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(int(r["TotalDurationNs"]) for r in rows)
print("== %s: %.1f ms kernel time, %d dispatches" % (sys.argv[1], tot / 1e6, sum(int(r["Calls"]) for r in rows)))
for r in sorted(rows, key=lambda r: -int(r["TotalDurationNs"]))[:8]:
    print("   %-60s %6s %9.2f ms" % (r["Name"][:60], r["Calls"], int(r["TotalDurationNs"]) / 1e6))
PY
done | tee gpurun_out/pipeprof_summary.txt
find gpurun_out/pipeprof -name "*kernel_trace.csv" -delete
