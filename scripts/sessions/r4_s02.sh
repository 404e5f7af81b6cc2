#!/bin/bash
# Round 4, GPU session 2: the FNO mixing paths at batch 1 / 8 / 32, the FNO block; A/B runs (LDS-staged FFT twiddles, the dftw load-batch depth, the 720 = 24 x 30 plan)
# and phase clocks of the FNO tail and the rfft2 passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
ROOT=$PWD
step() {
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "$ROOT/gpurun_out/$tag.log" | grep -v "warning: failed to meet" | tail -${TAILN:-12}
  if [ $rc -ne 0 ]; then echo "stopping: $tag failed ($rc)"; exit $rc; fi
}
# GEMM phase clocks (prologue / main loop / epilogue per workgroup) incl. the LN-fold fc1 and the statistics fc2
TAILN=60 step r4s02_gemm_stamps 200 ./variants/bin/gemm_stamps
TAILN=20 step r4s02_afno_stamps 200 ./variants/bin/afno_stamps
TAILN=8 step r4s02_fnomix 400 python -u bench/bench_fno_mix.py --rounds 3
TAILN=6 step r4s02_fno_b1 300 python -u bench/bench_fno.py --amd-only --rounds 6
# FNO block, this round (batched table setup, unit counters) vs the round-3 state (variants/r3), ABAB
for r in 1 2; do
  TAILN=2 step r4s02_fno_new_$r 200 python -u bench/bench_fno.py --amd-only --rounds 5
  (cd variants/r3 && TAILN=2 step r4s02_fno_old_$r 200 python -u bench/bench_fno.py --amd-only --rounds 5) || exit 1
done
# rfft2 / irfft2 720x1440: LDS-staged twiddles (variants/twlds = -DAMD_DFT_TW_LDS=1) vs the L1-table prefetch, ABAB
for r in 1 2; do
  step r4s01_fft_def_$r 200 python -u bench/bench_fft.py --rounds 8 --json gpurun_out/r4s01_fft_def_$r.json

  python3 -c "import json;d=json.load(open('gpurun_out/r4s01_fft_def_$r.json'));print('default', {k:round(d[k]['graph']['median_us'],2) for k in ('amd_rfft2','amd_irfft2')})"
  MI_DFT_LIB=$PWD/variants/twlds/_C.so step r4s01_fft_tw_$r 200 python -u bench/bench_fft.py --rounds 8 --json gpurun_out/r4s01_fft_tw_$r.json
  python3 -c "import json;d=json.load(open('gpurun_out/r4s01_fft_tw_$r.json'));print('twlds  ', {k:round(d[k]['graph']['median_us'],2) for k in ('amd_rfft2','amd_irfft2')})"
done
# FNO block: dftw_r2c with a wave's whole 1440-row share in one load batch (variants/dftwpf8) vs default, ABAB
for r in 1 2; do
  TAILN=2 step r4s01_fno_def_$r 200 python -u bench/bench_fno.py --amd-only --rounds 5
  MI_DFT_LIB=$PWD/variants/dftwpf8/_C.so TAILN=2 step r4s01_fno_pf8_$r 200 python -u bench/bench_fno.py --amd-only --rounds 5
done
# 720 = (24, 30) two-pass column / row plan vs (8, 9, 10): correctness, then rfft2 / irfft2 ABAB
MI_DFT_FFT_RADICES="720:24,30" TAILN=2 step r4s01_tests_2430 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_dft_gpu.py
for r in 1 2; do
  step r4s01_fft_d2_$r 200 python -u bench/bench_fft.py --rounds 8 --json gpurun_out/r4s01_fft_d2_$r.json
  python3 -c "import json;d=json.load(open('gpurun_out/r4s01_fft_d2_$r.json'));print('8,9,10 ', {k:round(d[k]['graph']['median_us'],2) for k in ('amd_rfft2','amd_irfft2')})"
  MI_DFT_FFT_RADICES="720:24,30" step r4s01_fft_2430_$r 200 python -u bench/bench_fft.py --rounds 8 --json gpurun_out/r4s01_fft_2430_$r.json
  python3 -c "import json;d=json.load(open('gpurun_out/r4s01_fft_2430_$r.json'));print('24,30  ', {k:round(d[k]['graph']['median_us'],2) for k in ('amd_rfft2','amd_irfft2')})"
done
# phase clocks of the fused FNO tail (fno_c2r_pw) and the rfft2 fixed passes (timing-only builds, variants/bin)
TAILN=30 step r4s01_fno_stamps 120 ./variants/bin/fno_stamps
TAILN=30 step r4s01_fft_stamps 120 ./variants/bin/fft_stamps
# fp32 FourCastNet step: AFNO C2R (split epilogue) with addends loaded 3 positions ahead at 3 WGs/CU
# (variants/c2rjit) vs all addends before the DFT at 2 WGs/CU (default), ABAB
for r in 1 2; do
  TAILN=1 step r4s02_step_def_$r 300 python -u bench.py --no-fft --extra-steps 0 --steps 10 --warmup 3
  MI_DFT_LIB=$PWD/variants/c2rjit/_C.so TAILN=1 step r4s02_step_jit_$r 300 python -u bench.py --no-fft --extra-steps 0 --steps 10 --warmup 3
done
