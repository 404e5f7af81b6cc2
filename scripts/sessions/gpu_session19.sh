#!/bin/bash
# GPU session 19 (round 3): (1) FNO block after the mixing-gather load batching (bf16 dftw on hi-only twiddles
# was tried and reverted: the standalone bf16 DFT op lost its ~1e-6 accuracy); (2) rfft2/irfft2 720x1440 A/B of the FFT radix plans: default (1440: 10,12,12 at 144 threads;
# 720 cols: 8,9,10 at 90 x 4) vs more threads per FFT (1440: 5,6,6,8 at 288; 720 cols: 4,4,5,9 at 180 x 4).
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
ALT="1440:5,6,6,8;720:4,4,5,9"
TAILN=3 step s19_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_fno.py tests/test_dft_gpu.py
TAILN=3 step s19_tests_alt 400 env MI_DFT_FFT_RADICES=$ALT python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_dft_gpu.py tests/test_engine.py
TAILN=3 step s19_fno 300 python -u bench/bench_fno.py --amd-only --rounds 10
for r in 1 2; do
  TAILN=2 step s19_fft_def_$r 300 python -u bench/bench_fft.py --rounds 10
  TAILN=2 step s19_fft_alt_$r 300 env MI_DFT_FFT_RADICES=$ALT python -u bench/bench_fft.py --rounds 10
  TAILN=2 step s19_fft_rows_$r 300 env MI_DFT_FFT_RADICES="1440:5,6,6,8" python -u bench/bench_fft.py --rounds 10
done
step s19_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fno19 -o fno -- python3 bench/bench_fno.py --amd-only --rounds 3
python3 scripts/kernel_summary.py gpurun_out/prof_fno19 > gpurun_out/prof_fno19.txt; head -8 gpurun_out/prof_fno19.txt
