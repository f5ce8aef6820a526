#!/bin/bash
# round 6: (1) the device name torch reports with and without rocprofv3 (the
# tuning keys carry it); (2) two benches at the driver's defaults with the
# committed seed table
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 120 python3 -c "import torch; print('plain:', repr(torch.cuda.get_device_name(0)), torch.cuda.get_device_properties(0).gcnArchName)" 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 rocprofv3 --kernel-trace -d /tmp/rp_name -o run -- python3 -c "import torch; print('rocprofv3:', repr(torch.cuda.get_device_name(0)), torch.cuda.get_device_properties(0).gcnArchName)" 2>&1 | grep -E "plain|rocprofv3:" | grep -v simple_timer
for i in 1 2; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench_r6_final_$i.json > gpurun_out/bench_r6_final_$i.log 2>&1 || exit $?
  python3 -c "
import json; j=json.load(open('gpurun_out/bench_r6_final_$i.json'))
print('run $i', j['value'], 'p50', j['p50_ms'], 'p99', j['p99_ms'], 'mi10', j['latency_mi10']['p50_ms'], j['latency_mi10']['p99_ms'], 'tuned', j['model_counters'].get('tune_tuned'), 'setup', j['timeline_s'].get('headline.setup'), 'lit2', j['literal']['config2_whole']['videos_per_s'], j['literal']['config2_whole_one_lane']['videos_per_s'], 'lit4', j['literal']['config4_segment']['videos_per_s'])"
done
