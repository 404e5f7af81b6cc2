#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
A="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
B="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA"
C="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
for s in A B C; do
  eval "P=\$$s"
  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv --pmc $P -d gpurun_out/pmcb_$s -o p -- python3 bench.py --steps 1 --warmup 0 --no-fft --no-graph --depth 2 > gpurun_out/pmcb_$s.log 2>&1 || { echo "pass $s failed"; tail -5 gpurun_out/pmcb_$s.log; }
done
python3 scripts/pmc_summary2.py gpurun_out/pmcb_A gpurun_out/pmcb_B gpurun_out/pmcb_C
