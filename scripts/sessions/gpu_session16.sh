#!/bin/bash
# GPU session 16 (round 3): FNO layer tail phase clocks + per-kernel ablation table (what bounds fno_c2r_pw).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 ./build_diag/fno_stamps > gpurun_out/s16_stamps.log 2>&1; rc=$?; cat gpurun_out/s16_stamps.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench/bench_kernels_fno.py > gpurun_out/s16_kern.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/s16_kern.log | tail -40; exit $rc
