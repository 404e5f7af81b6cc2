#!/bin/bash
# PMC counters (3 passes, kernel-trace only) for an arbitrary python command:
#   scripts/pmc_cmd.sh TAG script.py [args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
A="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
B="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA"
C="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
for s in A B C; do
  eval "P=\$$s"
  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv --pmc $P -d gpurun_out/pmc_${TAG}_$s -o p -- python3 "$@" > gpurun_out/pmc_${TAG}_$s.log 2>&1 || { echo "pass $s failed"; tail -5 gpurun_out/pmc_${TAG}_$s.log; exit 1; }
done
python3 scripts/pmc_summary2.py gpurun_out/pmc_${TAG}_A gpurun_out/pmc_${TAG}_B gpurun_out/pmc_${TAG}_C
