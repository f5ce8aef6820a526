#!/bin/bash
# PMC passes for one fp32 conv of the R(2+1)D-34 plan at several configs
# (kernel trace + counters only). LAYER, CFGS, CLIPS from the environment.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
LAYER=${LAYER:-conv2.blocks.0.conv1.spatial}
CFGS=${CFGS:-"1018 1050"}
CLIPS=${CLIPS:-128}
OUT=${OUT:-gpurun_out/pmc_r3}
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
for cfg in $CFGS; do
  i=0
  for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC" \
             "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT GRBM_GUI_ACTIVE" \
             "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    mkdir -p $OUT/c${cfg}; d=$OUT/c${cfg}/p$i
    timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $d -o run -- python scripts/conv_bench.py --dtype fp32 --clips $CLIPS --layer $LAYER --config $cfg --reps 3 > $d.log 2>&1
    rc=$?
    echo "cfg $cfg pass $i rc=$rc $(grep -h 'config' $d.log | tail -1)"
    if [ $rc -ne 0 ]; then tail -3 $d.log; fi
  done
  echo "== cfg $cfg"; KNAME=${KNAME:-conv_} python scripts/pmc_summary.py $OUT/c${cfg}
done
