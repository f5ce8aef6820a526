#!/bin/bash
# Build (CPU side: hipcc) and run the interprocess-event reproducer
# (csrc/bench/ipc_event_repro.cpp) on the GPU box.
#   bash scripts/ipc_event_repro.sh build      # here
#   bash scripts/ipc_event_repro.sh [rounds]   # GPU box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BIN=rnb_amd/_native/exp/ipc_event_repro
if [ "${1:-}" = "build" ]; then
  mkdir -p rnb_amd/_native/exp
  hipcc --offload-arch=gfx950 -O2 csrc/bench/ipc_event_repro.cpp -o $BIN; exit $?
fi
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 $BIN "${1:-2000}"
