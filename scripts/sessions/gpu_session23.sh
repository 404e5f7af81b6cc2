#!/bin/bash
# GPU session 23 (round 3): AFNO -O3 bisection, step 4 (vectorizer-off builds in diag_libs/): tw = both pass-1 twiddle
# reads 64-bit (control, fails in session 21); wait = the same + s_waitcnt lgkmcnt(0) right after every twiddle read;
# chk = the same + a volatile 32-bit re-read and compare (passed in session 22); three repeats each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2 3; do
for t in tw wait chk; do
  echo "== afno $t rep $rep"
  MI_DFT_LIB=$PWD/diag_libs/$t/_C.so timeout -k 10 300 python -u scripts/diag/afno_race_diag.py > gpurun_out/s23_afno_${t}_$rep.log 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/s23_afno_${t}_$rep.log | tail -2; [ $rc -eq 0 ] || { echo "afno $t ended abnormally ($rc)"; exit $rc; }
done
done
