#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_dft_gpu.py -q -x > gpurun_out/t_tune.log 2>&1; rc=$?; tail -3 gpurun_out/t_tune.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench/tune_fixed.py 2>&1 | grep -v amdgpu.ids || exit 1
TUNE_B=8 timeout -k 10 300 python bench/tune_fixed.py 2>&1 | grep -v amdgpu.ids || exit 1
bash scripts/pmc_fft.sh 2>&1 | grep -A1 "fixed"
