#!/bin/bash
# round 6 (final tree): per-dispatch MFMA / clock counters and per-family stall
# counters of one graphed 128-clip fp32 batch-BN forward (h3w in the set, seed picks)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1 RNB_TUNE_CACHE=gpurun_out/tune_pmc.json
rm -f $RNB_TUNE_CACHE
timeout -k 10 300 python3 scripts/bn_breakdown.py run --mode batch --clips 128 --reps 1 > gpurun_out/pmc_warm.log 2>&1 || { tail gpurun_out/pmc_warm.log; exit 1; }
d=gpurun_out/pmcf; rm -rf $d
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES \
  --kernel-trace --output-format csv -d $d -o run -- python3 scripts/bn_breakdown.py run --mode batch --clips 128 --reps 1 > $d.log 2>&1 || { tail $d.log; exit 1; }
python3 scripts/pmc_forward.py $d > gpurun_out/pmc_forward_128_r6.txt 2>&1
tail -22 gpurun_out/pmc_forward_128_r6.txt
rm -rf $d
for pass in A B; do
  if [ $pass = A ]; then C="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA";
  else C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum"; fi
  rm -rf gpurun_out/pmc$pass
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc$pass -o run \
    -- python3 scripts/bn_breakdown.py run --mode batch --clips 128 --reps 1 > gpurun_out/pmc$pass.log 2>&1 || { tail gpurun_out/pmc$pass.log; exit 1; }
done
python3 scripts/pmc_families.py gpurun_out/pmcA gpurun_out/pmcB > gpurun_out/pmc_families_128_r6.txt 2>&1
cat gpurun_out/pmc_families_128_r6.txt
rm -rf gpurun_out/pmcA gpurun_out/pmcB
