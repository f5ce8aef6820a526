#!/bin/bash
# round 5: same-box A/B of two builds of the kernels library on the conv2 /
# stem temporal layers: the in-tree one (cur) against
# rnb_amd/_native/exp/librnb_kernels_h3p_head.so (head: the committed h3p), alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
L=rnb_amd/_native/librnb_kernels.so
cp $L /tmp/lib_cur.so
for r in 1 2 3; do
  for v in cur head; do
    if [ $v = cur ]; then cp /tmp/lib_cur.so $L; else cp rnb_amd/_native/exp/librnb_kernels_h3p_head.so $L; fi
    timeout -k 10 200 python scripts/h3_layer_bench.py --clips 128 --cases k4,stemt --cids 1440 --rounds 3 > gpurun_out/libab_$v.txt 2>&1 || { tail gpurun_out/libab_$v.txt; cp /tmp/lib_cur.so $L; exit 1; }
    echo "$v round $r"; grep -v amdgpu.ids gpurun_out/libab_$v.txt
  done
done
cp /tmp/lib_cur.so $L
