#!/bin/bash
# GPU session 25 (round 3): AFNO -O3 bisection, step 6 (vectorizer-off builds in diag_libs/): asmpk (inline-asm
# ds_read_b64 + full wait + packed multiply with op_sel:[0,1], failed in session 24); asmnop = asmpk + 16 wait states
# between the wait and the packed multiply; asmr2 = asmpk with the pair read by ds_read2_b32.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2 3; do
for t in asmnop asmr2 asmpk; do
  echo "== afno $t rep $rep"
  MI_DFT_LIB=$PWD/diag_libs/$t/_C.so timeout -k 10 300 python -u scripts/diag/afno_race_diag.py > gpurun_out/s25_afno_${t}_$rep.log 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/s25_afno_${t}_$rep.log | tail -2; [ $rc -eq 0 ] || { echo "afno $t ended abnormally ($rc)"; exit $rc; }
done
done
# minimal-kernel attempt (scripts/diag/opsel_lds_repro.hip, built in the container): LDS-loaded pair -> v_pk_mul op_sel:[0,1]
for m in "0 77448 2944" "1 77448 2944" "2 77448 2944" "0 120000 2944" "0 16000 8192"; do
  timeout -k 10 120 ./diag_libs/opsel_lds_repro $m 200 || { echo "repro ended abnormally"; exit 1; }
done
