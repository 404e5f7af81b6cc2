#!/bin/bash
# Op-level timeline: roctx ranges (MI_DFT_TRACE=1: one per native op + one per AFNO block)
# with the kernels they launched, eager mode (ranges are host-side, a graph replay has none).
#   bash scripts/trace_bench.sh TAG   -> gpurun_out/trace_TAG/ (+ marker/kernel summary)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp MI_DFT_TRACE=1 HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${1:-trace}
timeout -k 10 600 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d gpurun_out/trace_$TAG -o t \
  -- python3 bench.py --steps 2 --warmup 1 --no-graph --no-fft --depth 2 > gpurun_out/trace_$TAG.log 2>&1
