#!/bin/bash
# Round 4, GPU session 12: rfft2 720x1440 with the row pass's intermediate written through L2 (variants/wt =
# -DAMD_DFT_R2C_WT=1: 16-B sc1 buffer stores, so the kernel boundary has no dirty intermediate to write back)
# vs the default, ABAB; the FFT GPU tests under the variant first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp MI_DFT_BOX_BUILD=0
ROOT=$PWD
WT=$PWD/variants/wt/_C.so
step() {
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "$ROOT/gpurun_out/$tag.log" | grep -v "warning: failed to meet" | tail -${TAILN:-12}
  if [ $rc -ne 0 ]; then echo "stopping: $tag failed ($rc)"; exit $rc; fi
}
MI_DFT_LIB=$WT TAILN=3 step r4s12_tests_wt 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dft_gpu.py
for r in 1 2 3; do
  step r4s12_fft_def_$r 200 python -u bench/bench_fft.py --rounds 8 --json gpurun_out/r4s12_fft_def_$r.json
  python3 -c "import json;d=json.load(open('gpurun_out/r4s12_fft_def_$r.json'));print('default', {k:round(d[k]['graph']['median_us'],2) for k in ('amd_rfft2','amd_irfft2')})"
  MI_DFT_LIB=$WT step r4s12_fft_wt_$r 200 python -u bench/bench_fft.py --rounds 8 --json gpurun_out/r4s12_fft_wt_$r.json
  python3 -c "import json;d=json.load(open('gpurun_out/r4s12_fft_wt_$r.json'));print('wt     ', {k:round(d[k]['graph']['median_us'],2) for k in ('amd_rfft2','amd_irfft2')})"
done
# bf16 AFNO spectral kernel at 4 workgroups per CU (variants/occ4 = -DAFNO_OCC96=4 -DAFNO_BPF=1: <= 128 VGPRs,
# 17 spilled) vs 3 (default): correctness, then the bf16 FourCastNet step, ABAB
OCC4=$PWD/variants/occ4/_C.so
MI_DFT_LIB=$OCC4 TAILN=3 step r4s12_tests_occ4 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_spectral_gpu.py
for r in 1 2; do
  TAILN=1 step r4s12_bf16_def_$r 300 python -u bench.py --no-fft --dtype bf16 --extra-steps 0 --steps 10 --warmup 3
  MI_DFT_LIB=$OCC4 TAILN=1 step r4s12_bf16_occ4_$r 300 python -u bench.py --no-fft --dtype bf16 --extra-steps 0 --steps 10 --warmup 3
done
