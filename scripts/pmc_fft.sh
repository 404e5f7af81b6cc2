#!/bin/bash
# rocprofv3 PMC passes over bench/bench_fft.py (rfft2/irfft2 720x1440 fp32): one run per
# counter group (never more than the per-block limits in one pass), then a per-kernel table.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
A="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
B="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM"
C="FETCH_SIZE"
D="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
for p in A B C D; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc ${!p} -d gpurun_out/pmc$p -o $p -- \
    python3 bench/bench_fft.py --rounds 1 --iters 5 > gpurun_out/pmc$p.log 2>&1 || exit $?
done
python3 scripts/pmc_summary.py gpurun_out/pmcA gpurun_out/pmcB gpurun_out/pmcC gpurun_out/pmcD
