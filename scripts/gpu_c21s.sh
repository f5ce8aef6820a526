# role-specialised fused (2+1)D kernel: exact tests, bottleneck table, per-layer table, bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv21.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/c21_tests.log 2>&1; rc=$?
tail -3 gpurun_out/c21_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/c21_exp.py run --clips 128 > gpurun_out/c21_exp.txt 2>&1 || exit $?
cat gpurun_out/c21_exp.txt
timeout -k 10 300 python scripts/profile_layers.py --depth 34 --clips 128 --autotune --fuse > gpurun_out/layers128_fused.txt 2>&1 || exit $?
grep -E "conv2\.|TOTAL" gpurun_out/layers128_fused.txt
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
