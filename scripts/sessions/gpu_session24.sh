#!/bin/bash
# GPU session 24 (round 3): AFNO -O3 bisection, step 5 (vectorizer-off builds in diag_libs/): the 64-bit pass-1 twiddle
# reads as inline-asm ds_read_b64 + s_waitcnt lgkmcnt(0), consumed by an unpacked scalar fp32 multiply (asmsc) or by
# the packed v_pk_mul/v_pk_fma multiply (asmpk); tw (plain 64-bit reads, fails in sessions 21-23) as the control.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2 3; do
for t in asmsc asmpk tw; do
  echo "== afno $t rep $rep"
  MI_DFT_LIB=$PWD/diag_libs/$t/_C.so timeout -k 10 300 python -u scripts/diag/afno_race_diag.py > gpurun_out/s24_afno_${t}_$rep.log 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/s24_afno_${t}_$rep.log | tail -2; [ $rc -eq 0 ] || { echo "afno $t ended abnormally ($rc)"; exit $rc; }
done
done
