set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/mfma_split.py > gpurun_out/mfma_split.txt 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench0.log 2>&1
rc=$?; tail -3 gpurun_out/bench0.log; cat gpurun_out/mfma_split.txt; exit $rc
