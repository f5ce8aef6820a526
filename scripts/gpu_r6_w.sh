#!/bin/bash
# round 6: three-stage h3 direct configs (ids 1313-1316) -- GPU tests of every
# h3 config, then the layer table of the shapes the h3 direct family carries
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_h3.py > gpurun_out/w_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/w_tests.log; exit 1; }
tail -2 gpurun_out/w_tests.log
timeout -k 10 600 python3 scripts/h3_layer_bench.py --clips 128 --only-h3 \
  --cases k6,k8,k11,k12,k14,k17,k18,k20 > gpurun_out/w_layers_128.txt 2>&1 || { echo "layers 128 failed"; tail gpurun_out/w_layers_128.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/w_layers_128.txt | awk '{print}' | head -200 > /dev/null
timeout -k 10 400 python3 scripts/h3_layer_bench.py --clips 16 --only-h3 \
  --cases k8,k12,k14,k18,k20 > gpurun_out/w_layers_16.txt 2>&1 || { echo "layers 16 failed"; tail gpurun_out/w_layers_16.txt; exit 1; }
for f in gpurun_out/w_layers_128.txt gpurun_out/w_layers_16.txt; do
  python3 - "$f" <<'PY'
import sys, collections
best = collections.OrderedDict()
for line in open(sys.argv[1]):
    p = line.split()
    if len(p) < 6 or p[2] != "cid":
        continue
    case, cid, ms = p[0], int(p[3]), float(p[4])
    best.setdefault(case, []).append((ms, cid))
for case, v in best.items():
    v.sort()
    new = [x for x in v if 1313 <= x[1] <= 1316]
    print(sys.argv[1].split('_')[-1], case, "best", v[:3], "best-new", new[:1])
PY
done
