#!/bin/bash
# GPU session 21 (round 3): full GPU tier on the new defaults (1440 plan (5,6,6,8) at 288 threads, 20-channel
# mixing-gather batches), FFT + FNO benches, and the AFNO -O3 bisection continued: the tw build (vectorizer off,
# pass-1 twiddles read as 64-bit LDS loads from the top of the dynamic allocation) with extra unused LDS
# allocated behind the table (MI_DFT_AFNO_LDS_EXTRA), and the vectorizer-on build (vec1) likewise.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "gpurun_out/$tag.log" | grep -v "warning: failed to meet" | tail -${TAILN:-12}
  if [ $rc -ne 0 ]; then echo "stopping: $tag failed ($rc)"; exit $rc; fi
}
for cfg in "tw:0" "tw:512" "tw:4096" "vec1:512"; do
  t=${cfg%%:*}; x=${cfg#*:}
  echo "== afno $t extra=$x"
  MI_DFT_AFNO_LDS_EXTRA=$x MI_DFT_LIB=$PWD/diag_libs/$t/_C.so timeout -k 10 300 python -u scripts/diag/afno_race_diag.py \
    > gpurun_out/s21_afno_${t}_$x.log 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/s21_afno_${t}_$x.log; [ $rc -eq 0 ] || { echo "afno ended abnormally ($rc)"; exit $rc; }
done
TAILN=4 step s21_tests 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests
TAILN=2 step s21_fft_1 300 python -u bench/bench_fft.py --rounds 10
TAILN=2 step s21_fft_2 300 python -u bench/bench_fft.py --rounds 10
TAILN=3 step s21_fno 300 python -u bench/bench_fno.py --amd-only --rounds 10
TAILN=3 step s21_bench 600 python -u bench.py
