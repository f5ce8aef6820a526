# bench.py at driver defaults + per-layer table (128 clips, autotuned)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --trace gpurun_out/bench_kernels.txt > gpurun_out/bench.log 2>&1; rc=$?
tail -3 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/profile_layers.py --depth 34 --clips 128 --autotune > gpurun_out/layers128.txt 2>&1; rc=$?
tail -3 gpurun_out/layers128.txt
exit $rc
