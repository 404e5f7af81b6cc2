#!/bin/bash
# rocprofv3 PMC passes over bench/pmc_targets.py (FFT row/column kernels, FNO block, FourCastNet
# fp32 + bf16 block kernels and GEMMs): one run per counter group, each within the per-block
# counter limits, kernel trace only.  Usage: bash scripts/pmc_targets.sh TAG [pmc_targets args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
B="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA"
C="FETCH_SIZE"
D="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
for p in A B C D; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc ${!p} -d gpurun_out/pmc_${TAG}_$p -o $p -- \
    python3 bench/pmc_targets.py "$@" > gpurun_out/pmc_${TAG}_$p.log 2>&1 || { echo "pass $p failed"; tail -5 gpurun_out/pmc_${TAG}_$p.log; exit 1; }
  echo "pass $p ok"
done
python3 scripts/pmc_table.py gpurun_out/pmc_${TAG}_A gpurun_out/pmc_${TAG}_B gpurun_out/pmc_${TAG}_C gpurun_out/pmc_${TAG}_D \
  > gpurun_out/pmc_${TAG}_table.txt
cat gpurun_out/pmc_${TAG}_table.txt
