# 2-rank bench rehearsal on one GPU (gloo, shared device) + launcher pipeline configs
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 env RNB_BENCH_BACKEND=gloo RNB_BENCH_SHARE_GPU=1 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
    bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/bench_2rank_shared.log 2>&1 || exit $?
tail -1 gpurun_out/bench_2rank_shared.log
bash scripts/gpu_pipelines.sh > gpurun_out/pipelines_run.log 2>&1 || exit $?
tail -30 gpurun_out/pipelines_run.log
