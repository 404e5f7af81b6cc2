#!/bin/bash
# GPU CI on the MI355X box (reference: build_with_docker.sh runs `pip install -e . && pytest .`):
# build in-tree for gfx950, then the CPU and GPU tiers, each under its own time limit.
#   gpurun --timeout 1200 -- bash scripts/ci_gpu.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m tensorrt_dft_plugins_amd._build > gpurun_out/ci_build.log 2>&1 || { tail -20 gpurun_out/ci_build.log; exit 1; }
timeout -k 10 600 python -m pytest tests -q -m "not gpu" -x > gpurun_out/ci_cpu.log 2>&1 || { tail -20 gpurun_out/ci_cpu.log; exit 1; }
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/ci_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/ci_cpu.log gpurun_out/ci_gpu.log
exit $rc
