#!/bin/bash
# GPU tier after the fused-x3 / IPC changes + FFT column-pass study (rfft2 cfg x XCD, PMC).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S=scripts/gpu_step.sh
bash $S fftcfg 300 python3 -u bench/bench_fft_cfg.py auto 90,4 90,8 45,8 45,16 || exit $?
bash $S gputests 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
bash $S pmcfft 420 bash scripts/pmc_fft.sh || exit $?
PROF_TAG=_r2g bash $S profbench 400 bash scripts/prof_bench.sh || exit $?
