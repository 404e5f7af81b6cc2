#!/bin/bash
# GPU session 15 (round 3): per-kernel tables of the FNO block (config 3) and of rfft2/irfft2 720x1440 (config 2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fno -o fno -- \
  python3 bench/bench_fno.py --amd-only --rounds 3 > gpurun_out/prof_fno.log 2>&1 || { tail -5 gpurun_out/prof_fno.log; exit 1; }
python3 scripts/kernel_summary.py gpurun_out/prof_fno
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fft -o fft -- \
  python3 bench/bench_fft.py --rounds 3 > gpurun_out/prof_fft.log 2>&1 || { tail -5 gpurun_out/prof_fft.log; exit 1; }
python3 scripts/kernel_summary.py gpurun_out/prof_fft
