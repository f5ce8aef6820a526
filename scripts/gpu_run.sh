#!/bin/bash
# One GPU-box session made of named steps, run in order; each GPU step has
# its own time limit and a crash / abort / timeout (rc not 0 or 1) stops the
# script. Logs go to gpurun_out/<step>.log.
#
#   bash scripts/gpu_run.sh tests bench:20 layers:128 x6exp pmc:conv2.blocks.0.conv1.spatial:1018,1050
#
# steps:
#   build                 python -m rnb_amd.build
#   tests[:FILTER]        pytest -m gpu (optional -k FILTER)
#   smoke                 __graft_entry__.smoke()
#   bench[:STEPS]         bench.py at the driver defaults (JSON in gpurun_out/bench.json)
#   benchargs:ARGS        bench.py with extra arguments (commas -> spaces)
#   layers[:CLIPS]        per-conv table of the fp32 R(2+1)D-34 forward (autotuned)
#   wino[:CLIPS]          every Winograd variant per layer shape (fp32)
#   x6exp                 x6 Winograd bottleneck experiments (scripts/x6_exp.py)
#   x6dexp                x6 direct-conv bottleneck experiments (scripts/x6d_exp.py)
#   bnbreak[:CLIPS]       kernel breakdown of one graphed batch-BN forward (rocprofv3)
#   pmc:LAYER:CFGS        per-dispatch PMC passes of one conv (scripts/gpu_pmc_conv.sh)
#   fold:N                bench.py --gpus N through torchrun, all ranks folded onto GPU 0
#   mfma                  MFMA rate / split-bf16 numerics microbenchmark
#   repro[:ROUNDS]        interprocess-event wait reproducer (csrc/bench/ipc_event_repro.cpp)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
run() {  # run <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n "${TAIL:-15}" "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for step in "$@"; do
  name=${step%%:*}
  arg=""; [ "$name" != "$step" ] && arg=${step#*:}
  case $name in
    build) run build 600 python -m rnb_amd.build ;;
    tests)
      if [ -n "$arg" ]; then
        run tests 1100 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 \
          --timeout-method thread -k "$arg"
      else
        run tests 1100 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 \
          --timeout-method thread
      fi ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py --steps "${arg:-10}" --warmup 2 \
             --json-out gpurun_out/bench.json ;;
    benchargs) run benchargs 900 python bench.py ${arg//,/ } --json-out gpurun_out/benchargs.json ;;
    layers) run layers 400 python scripts/profile_layers.py --depth 34 --clips "${arg:-128}" \
              --dtype fp32 --autotune ;;
    wino) run wino 400 python scripts/profile_layers.py --depth 34 --clips "${arg:-128}" \
            --dtype fp32 --list-wino --reps 5 ;;
    x6exp) run x6exp 300 python -u scripts/x6_exp.py run ;;
    x6dexp) run x6dexp 300 python -u scripts/x6d_exp.py run ;;
    x6dsweep) run x6dsweep 300 python -u scripts/x6d_exp.py sweep ;;
    x6dsmall) run x6dsmall 300 python -u scripts/x6d_exp.py small ;;
    bnbreak)
      rm -rf gpurun_out/bnbreak
      run bnbreak 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bnbreak -o run \
        -- python3 scripts/bn_breakdown.py run --mode batch --clips "${arg:-128}"
      trace=$(ls gpurun_out/bnbreak/*/*/run_kernel_trace.csv gpurun_out/bnbreak/*/run_kernel_trace.csv \
                 gpurun_out/bnbreak/run_kernel_trace.csv 2>/dev/null | tail -1)
      [ -n "$trace" ] && python3 scripts/bn_breakdown.py parse "$trace" --kernels 12 \
        > gpurun_out/bnbreak.txt && head -n 40 gpurun_out/bnbreak.txt ;;
    pmc) layer=${arg%%:*}; cfgs=${arg#*:}
         LAYER=$layer CFGS="${cfgs//,/ }" run pmc 900 bash scripts/gpu_pmc_conv.sh ;;
    fold) n=${arg:-2}
          # torchrun ranks coordinate through the store (no GPU open); the
          # launcher on rank 0 runs n loaders + n runners folded onto GPU 0
          export RNB_FOLD_GPUS=1
          run fold$n 900 python -m torch.distributed.run --nnodes=1 \
            --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port 29631 bench.py \
            --gpus "$n" --steps 4 --warmup 1 --replicas 1 --loaders 1 \
            --json-out gpurun_out/fold$n.json
          unset RNB_FOLD_GPUS ;;
    foldl) n=${arg:-8}
          # the same topology from one bench process (no torchrun ranks)
          export RNB_FOLD_GPUS=1
          run foldl$n 900 python bench.py --gpus "$n" --steps 4 --warmup 1 --replicas 1 \
            --loaders 1 --json-out gpurun_out/foldl$n.json
          unset RNB_FOLD_GPUS ;;
    repro) run repro 150 bash scripts/ipc_event_repro.sh "${arg:-2000}" ;;
    mfma) run mfma 120 python -u scripts/mfma_split.py ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
