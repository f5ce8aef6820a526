#!/bin/bash
# round 5: geometric buckets + tuning snapped to the buckets holding 64 / 128
# clips, against the exact-power-of-two tuning and 4-clip buckets, 20 steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python scripts/ab_bench.py --rounds 2 --out gpurun_out/ab_snap.txt \
  "geosnap||--steps 20" "geopow2|RNB_TUNE_SNAP=0|--steps 20" "step4||--steps 20 --bucket-step 4"
rc=$?; cat gpurun_out/ab_snap.txt
for f in gpurun_out/ab_geosnap_*.json gpurun_out/ab_geopow2_*.json gpurun_out/ab_step4_*.json; do
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['timeline_s'].get('headline.setup'))" $f
done
exit $rc
