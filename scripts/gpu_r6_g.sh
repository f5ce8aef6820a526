#!/bin/bash
# round 6: PMC passes of conv2 spatial (128 clips) on the Winograd h3 kernel
# (1460) against the row-band h3q config (1387)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LAYER=conv2.blocks.0.conv1.spatial CFGS="1460 1387" CLIPS=128 OUT=gpurun_out/pmc_h3w \
  bash scripts/gpu_pmc_conv.sh > gpurun_out/pmc_h3w.log 2>&1
rc=$?; tail -60 gpurun_out/pmc_h3w.log; exit $rc
