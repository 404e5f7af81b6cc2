#!/bin/bash
# Round 4, GPU session 18: the head GEMM's un-patchify epilogue staged through LDS (whole-line stores) vs the
# scatter straight from the MFMA layout (variants/direct = -DGEMM_UNPATCH_STAGED=0): tests, then both steps ABAB.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp MI_DFT_BOX_BUILD=0
ROOT=$PWD
V=$PWD/variants/direct/_C.so
step() {
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "$ROOT/gpurun_out/$tag.log" | grep -v "warning: failed to meet" | tail -${TAILN:-12}
  if [ $rc -ne 0 ]; then echo "stopping: $tag failed ($rc)"; exit $rc; fi
}
TAILN=3 step r4s18_tests 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_patch_gemm.py \
  tests/test_models.py tests/test_spectral_gpu.py tests/test_fp32_path.py tests/test_gemm.py
for r in 1 2; do
  TAILN=1 step r4s18_new_$r 300 python -u bench.py --no-fft --steps 10 --warmup 3
  MI_DFT_LIB=$V TAILN=1 step r4s18_old_$r 300 python -u bench.py --no-fft --steps 10 --warmup 3
done
PROF_TAG=_r4s18 TAILN=12 step r4s18_prof 400 bash scripts/prof_bench.sh
