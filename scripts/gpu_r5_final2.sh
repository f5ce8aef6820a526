#!/bin/bash
# round 5 verification with the in-tree libraries (no rebuild): whole GPU suite,
# smoke, forward breakdowns at 128 and 1 clip, one bench at the driver's defaults
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
trace_of() { ls $1/*/*/run_kernel_trace.csv $1/*/run_kernel_trace.csv $1/run_kernel_trace.csv 2>/dev/null | tail -1; }
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 6 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for c in 128 1; do
  d=gpurun_out/bnb_$c; rm -rf $d
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
    -- python3 scripts/bn_breakdown.py run --mode batch --clips $c > $d.log 2>&1 || { echo "bnb $c failed"; tail $d.log; exit 1; }
  python3 scripts/bn_breakdown.py parse "$(trace_of $d)" --kernels 18 > gpurun_out/bnb_$c.txt
  head -14 gpurun_out/bnb_$c.txt
  rm -rf $d
done
step bench 600 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_final2.json
