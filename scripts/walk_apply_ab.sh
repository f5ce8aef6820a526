#!/bin/bash
# A/B of the one-dispatch BN walk + apply (RNB_BN_WALK_APPLY=1) against the
# walk + apply pair (=0): graphed batch-BN forwards at small buckets, one
# process per run, interleaved over rounds, one shared tuning cache (the
# first run of a bucket tunes it).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0 RNB_TUNE_CACHE=/tmp/wa_tune.json
for clips in ${CLIPS:-4 8 16 32}; do
  for rnd in 1 2 3; do
    for mode in 1 0; do
      out=$(RNB_BN_WALK_APPLY=$mode timeout -k 10 300 python scripts/bn_breakdown.py run \
              --mode batch --clips $clips --reps 50 2>&1 | grep "per graphed") || exit 1
      echo "clips $clips round $rnd walk_apply=$mode: $out"
    done
  done
done
