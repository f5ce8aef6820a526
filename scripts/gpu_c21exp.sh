# fused (2+1)D kernel bottleneck table + rocprofv3 kernel stats of the bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python scripts/c21_exp.py run --clips 128 > gpurun_out/c21_exp.txt 2>&1 || exit $?
cat gpurun_out/c21_exp.txt
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 10 --warmup 2 > gpurun_out/rocprof_bench.log 2>&1 || exit $?
tail -1 gpurun_out/rocprof_bench.log
find gpurun_out/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -25 {}'
