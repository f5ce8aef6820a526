#!/bin/bash
# bench.py at several argument sets (';'-separated in SWEEP_ARGS; an empty
# entry = the defaults), one line per run: videos/s, Poisson p50 / p99 ms,
# job wall s. Extras and the numerics check are off to keep runs short.
#   SWEEP_ARGS=";--clips-per-batch 256 --video-batch 128" bash scripts/bench_args_sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
IFS=";" read -ra SW <<< "${SWEEP_ARGS:-;--clips-per-batch 256 --video-batch 128}"
i=0
for args in "${SW[@]}"; do
  i=$((i + 1))
  echo "=== run $i args: $args"
  log=gpurun_out/sw$i.log
  # the bench prints little while it tunes: a heartbeat keeps the call alive
  ( while sleep 60; do echo "  ... $(date +%T) $(wc -l < $log 2>/dev/null) lines"; done ) &
  hb=$!
  # an entry may start with ENV=VALUE words (exported for that run only)
  envs=(); rest=()
  for w in $args; do
    if [[ ${#rest[@]} -eq 0 && $w == *=* && $w != --* ]]; then envs+=("$w"); else rest+=("$w"); fi
  done
  env "${envs[@]}" timeout -k 10 600 python bench.py --steps "${STEPS:-20}" --warmup 2 \
    --no-literal --no-check "${rest[@]}" > $log 2>&1
  rc=$?
  kill $hb 2>/dev/null
  grep -h '"metric"' $log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['p50_ms'], d['p99_ms'], d['config']['job_wall_s'])"
  if [ $rc -ne 0 ]; then tail -5 $log; exit $rc; fi
done
