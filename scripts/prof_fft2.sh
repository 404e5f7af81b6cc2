#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench/ablate_fft.py > gpurun_out/ablate.log 2>&1 || exit $?
cat gpurun_out/ablate.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY -d gpurun_out/pmc_fft -o pmc -- python3 bench/bench_fft.py --rounds 1 --iters 5 > gpurun_out/pmc_fft.log 2>&1 || exit $?
ls gpurun_out/pmc_fft
