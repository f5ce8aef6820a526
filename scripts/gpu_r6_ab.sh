#!/bin/bash
# round 6: re-tune every bench shape with more timing (4 alternating rounds,
# >= 2 ms per timing) into a fresh cache, then A/B that cache as the seed
# against the committed seed table (separate job caches, 3 interleaved rounds)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
rm -f gpurun_out/tune_r6b.json /tmp/tc_old.json /tmp/tc_new.json
RNB_TUNE_SEED=0 RNB_TUNE_ROUNDS=4 RNB_TUNE_MIN_MS=2 RNB_TUNE_CACHE=$PWD/gpurun_out/tune_r6b.json \
  timeout -k 10 900 python bench.py --steps 4 --warmup 1 --no-check --json-out gpurun_out/bench_retune.json \
  > gpurun_out/bench_retune.log 2>&1 || { echo "retune failed"; tail -20 gpurun_out/bench_retune.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/tune_r6b.json')); s=json.load(open('rnb_amd/ops/tune_seed.json'))['entries']
same=sum(1 for k,v in d.items() if s.get(k)==v); print('retuned shapes', len(d), 'same pick as the seed', same)
j=json.load(open('gpurun_out/bench_retune.json')); print('retune setup', j['timeline_s'].get('headline.setup'))"
timeout -k 10 1300 python scripts/ab_bench.py --rounds 3 --steps 10 --timeout 300 \
  --out gpurun_out/ab_retune.txt \
  "seed|RNB_TUNE_CACHE=/tmp/tc_old.json|" \
  "retune|RNB_TUNE_CACHE=/tmp/tc_new.json,RNB_TUNE_SEED=$PWD/gpurun_out/tune_r6b.json|"
