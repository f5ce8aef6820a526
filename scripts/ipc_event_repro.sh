#!/bin/bash
# Build and run the interprocess-event reproducer
# (csrc/bench/ipc_event_repro.cpp). The binary is built from source into
# build/ (git-ignored), never committed.
#   bash scripts/ipc_event_repro.sh build      # here or on the GPU box
#   bash scripts/ipc_event_repro.sh [rounds]   # GPU box (builds first if missing)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BIN=build/exp/ipc_event_repro
build() { mkdir -p build/exp && hipcc --offload-arch=gfx950 -O2 csrc/bench/ipc_event_repro.cpp -o $BIN; }
if [ "${1:-}" = "build" ]; then build; exit $?; fi
[ -x $BIN ] || build || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 $BIN "${1:-2000}"
