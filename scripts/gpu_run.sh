#!/bin/bash
# One GPU-box session made of named steps, run in order; each GPU step has
# its own time limit and a crash / abort / timeout (rc not 0 or 1) stops the
# script. Logs go to gpurun_out/<step>.log.
#
#   bash scripts/gpu_run.sh tests bench:20 layers:128 pmc:conv2.blocks.0.conv1.spatial:1018,1050
#
# steps:
#   build                 python -m rnb_amd.build
#   tests[:FILTER]        pytest -m gpu (optional -k FILTER)
#   smoke                 __graft_entry__.smoke()
#   bench[:STEPS]         bench.py at the driver defaults (JSON in gpurun_out/bench.json)
#   benchargs:ARGS        bench.py with extra arguments (commas -> spaces)
#   layers[:CLIPS]        per-conv table of the fp32 R(2+1)D-34 forward (autotuned)
#   wino[:CLIPS]          every Winograd variant per layer shape (fp32)
#   compare[:CLIPS]       per conv: the best config of each kernel family (fp32 / wino / x6 / h3)
#   bnbreak[:CLIPS]       kernel breakdown of one graphed batch-BN forward (rocprofv3)
#   pmc:LAYER:CFGS        per-dispatch PMC passes of one conv (scripts/gpu_pmc_conv.sh)
#   fold:N                bench.py --gpus N through torchrun, all ranks folded onto GPU 0
#   mfma                  MFMA rate / split-bf16 numerics microbenchmark
#   repro[:ROUNDS]        interprocess-event wait reproducer (csrc/bench/ipc_event_repro.cpp)
#   ipcmatrix[:ROUNDS]    which factor decides the IPC-event wait (scripts/ipc_event_matrix.py)
#   ipcscale              16 rings x 386 slots in one consumer (tests/test_gpu_ipc_scale.py)
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
    compare) run compare 600 python scripts/profile_layers.py --depth 34 --clips "${arg:-128}" \
               --dtype fp32 --compare --reps 5 ;;
    bnbreak)
      c=${arg:-128}
      rm -rf gpurun_out/bnbreak_$c
      run bnbreak 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bnbreak_$c -o run \
        -- python3 scripts/bn_breakdown.py run --mode batch --clips "$c"
      trace=$(ls gpurun_out/bnbreak_$c/*/*/run_kernel_trace.csv gpurun_out/bnbreak_$c/*/run_kernel_trace.csv \
                 gpurun_out/bnbreak_$c/run_kernel_trace.csv 2>/dev/null | tail -1)
      [ -n "$trace" ] && python3 scripts/bn_breakdown.py parse "$trace" --kernels 40 \
        > gpurun_out/bnbreak_$c.txt && head -n 60 gpurun_out/bnbreak_$c.txt ;;
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
    ipcmatrix) run ipcmatrix 400 python -u scripts/ipc_event_matrix.py --rounds "${arg:-200}" \
                 --out gpurun_out/ipc_event_matrix.txt ;;
    ipcscale) run ipcscale 300 python -u -m pytest tests/test_gpu_ipc_scale.py -v -s \
                -p no:cacheprovider --timeout 240 --timeout-method thread ;;
    mfma) run mfma 120 python -u scripts/mfma_split.py ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
