# halows (weight-stationary conv2 spatial) check: exact tests, A/B timing, bottleneck variants
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k halo -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ws_tests.log 2>&1; rc=$?
tail -5 gpurun_out/ws_tests.log
[ $rc -ne 0 ] && exit $rc
for cfg in 102 104 102 104; do
  timeout -k 10 120 python scripts/conv_bench.py --layer conv2.blocks.0.conv1.spatial --clips 128 --config $cfg --reps 20 || exit $?
done
timeout -k 10 300 python scripts/kernel_exp.py run --clips 128 --layers conv2.blocks.0.conv1.spatial --configs 102,104
