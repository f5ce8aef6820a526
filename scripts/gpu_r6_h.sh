#!/bin/bash
# round 6: PMC passes of conv2 spatial (128 clips) on the second h3w build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LAYER=conv2.blocks.0.conv1.spatial CFGS="1460" CLIPS=128 OUT=gpurun_out/pmc_h3w2 KNAME=conv_h3w \
  bash scripts/gpu_pmc_conv.sh > gpurun_out/pmc_h3w2.log 2>&1
rc=$?; tail -32 gpurun_out/pmc_h3w2.log; exit $rc
