#!/bin/bash
# Round 4, GPU session 7: the two-phase GEMM main loop (variants/half = -DGEMM_HALF=3: 32 / 48 MFMAs per
# section, wave group 1 fills the B regions) -- correctness, bf16 GEMMs vs hipBLASLt, bf16x3 GEMMs, phase
# clocks, and the FourCastNet step, each ABAB against the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp MI_DFT_BOX_BUILD=0
ROOT=$PWD
HALF=$PWD/variants/half/_C.so
step() {
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "$ROOT/gpurun_out/$tag.log" | grep -v "warning: failed to meet" | tail -${TAILN:-12}
  if [ $rc -ne 0 ]; then echo "stopping: $tag failed ($rc)"; exit $rc; fi
}
MI_DFT_LIB=$HALF TAILN=4 step r4s07_tests_half 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gemm.py tests/test_gemm_variants.py tests/test_fp32_path.py tests/test_patch_gemm.py tests/test_models.py
TAILN=40 step r4s07_stamps_half 200 ./variants/bin/gemm_stamps_half
TAILN=40 step r4s07_stamps_def 200 ./variants/bin/gemm_stamps
for r in 1 2; do
  TAILN=10 step r4s07_bf16_def_$r 300 python -u bench/bench_gemm.py --rounds 3
  MI_DFT_LIB=$HALF TAILN=10 step r4s07_bf16_half_$r 300 python -u bench/bench_gemm.py --rounds 3
done
for r in 1 2; do
  TAILN=10 step r4s07_x3_def_$r 300 python -u bench/bench_gemm.py --x3 --rounds 3
  MI_DFT_LIB=$HALF TAILN=10 step r4s07_x3_half_$r 300 python -u bench/bench_gemm.py --x3 --rounds 3
done
for r in 1 2; do
  TAILN=1 step r4s07_step_def_$r 300 python -u bench.py --no-fft --steps 10 --warmup 3
  MI_DFT_LIB=$HALF TAILN=1 step r4s07_step_half_$r 300 python -u bench.py --no-fft --steps 10 --warmup 3
done
