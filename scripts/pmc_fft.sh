#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
A="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
B="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc $A -d gpurun_out/pmcA -o a -- python3 bench/bench_fft.py --rounds 1 --iters 5 > gpurun_out/pmcA.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc $B -d gpurun_out/pmcB -o b -- python3 bench/bench_fft.py --rounds 1 --iters 5 > gpurun_out/pmcB.log 2>&1 || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmcA gpurun_out/pmcB
