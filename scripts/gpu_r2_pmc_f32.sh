#!/bin/bash
# fp32 conv kernel counters (one pass per counter group; kernel trace + pmc
# only) and a rocprofv3 kernel-stats table of the single-process fp32 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${OUT:-gpurun_out/pmc_f32}
mkdir -p $OUT
LAYER=${LAYER:-conv2.blocks.0.conv1.spatial}
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/p$i -o run -- python scripts/conv_bench.py --dtype fp32 --clips ${CLIPS:-64} --layer $LAYER --reps 5 ${CONFIG:+--config $CONFIG} > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"; tail -2 $OUT/p$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
KNAME=${KNAME:-conv_f32} python scripts/pmc_summary.py $OUT | tee $OUT/summary.txt
[ -n "${SKIP_BENCH:-}" ] && exit 0
rm -rf gpurun_out/prof_f32
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f32 -o run -- python bench.py --pipeline fused --dtype fp32 --steps 5 --warmup 1 > gpurun_out/prof_f32.log 2>&1
rc=$?
echo "rocprof bench rc=$rc"; tail -1 gpurun_out/prof_f32.log | cut -c1-300
f=$(find gpurun_out/prof_f32 -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && head -30 "$f" | cut -d, -f1-8
exit $rc
