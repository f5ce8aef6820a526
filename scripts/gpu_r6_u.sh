#!/bin/bash
# round 6: A/B of the BN tail and the split-K fix-up on the graphed forward
# (plain wall time per forward, interleaved settings, seed-table picks)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
out=gpurun_out/ab_tail.txt; : > $out
for rnd in 1 2; do
  for c in 1 4 16; do
    for s in "0 0" "0 2048" "1 0" "1 2048"; do
      set -- $s
      r=$(RNB_SPLITK_FIXUP=$1 RNB_BN_TAIL_MAX=$2 timeout -k 10 200 python3 scripts/bn_breakdown.py run --mode batch --clips $c --reps 200 2>&1 | tail -1) || { echo "run failed: $r"; exit 1; }
      echo "round $rnd clips $c fixup $1 tail $2: $r" | tee -a $out
    done
  done
done
