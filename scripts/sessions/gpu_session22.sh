#!/bin/bash
# GPU session 22 (round 3): AFNO -O3 bisection, step 3.  Vectorizer-off builds (diag_libs/, built in the container):
#   fwd: only the forward FFT_H pass-1 twiddles read as 64-bit LDS loads; inv: only the inverse pass 1;
#   chk: both, each 64-bit read re-read as two volatile 32-bit loads, a mismatch poisons the butterfly with NaN.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for t in fwd inv chk; do
  echo "== afno $t"
  MI_DFT_LIB=$PWD/diag_libs/$t/_C.so timeout -k 10 300 python -u scripts/diag/afno_race_diag.py > gpurun_out/s22_afno_$t.log 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/s22_afno_$t.log; [ $rc -eq 0 ] || { echo "afno $t ended abnormally ($rc)"; exit $rc; }
done
