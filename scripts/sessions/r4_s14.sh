#!/bin/bash
# Round 4, GPU session 14: bf16x3 MFMA order A/B -- the three products of one accumulator tile back to back
# (variants/x3tile = -DGEMM_X3_TILE=1: fragments reused by consecutive MFMAs) vs products outermost (default).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp MI_DFT_BOX_BUILD=0
ROOT=$PWD
V=$PWD/variants/x3tile/_C.so
step() {
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "$ROOT/gpurun_out/$tag.log" | grep -v "warning: failed to meet" | tail -${TAILN:-12}
  if [ $rc -ne 0 ]; then echo "stopping: $tag failed ($rc)"; exit $rc; fi
}
MI_DFT_LIB=$V TAILN=3 step r4s14_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm.py tests/test_gemm_variants.py tests/test_fp32_path.py
for r in 1 2; do
  TAILN=6 step r4s14_x3_def_$r 300 python -u bench/bench_gemm.py --x3 --rounds 3
  MI_DFT_LIB=$V TAILN=6 step r4s14_x3_tile_$r 300 python -u bench/bench_gemm.py --x3 --rounds 3
done
for r in 1 2; do
  TAILN=1 step r4s14_step_def_$r 300 python -u bench.py --no-fft --extra-steps 0 --steps 10 --warmup 3
  MI_DFT_LIB=$V TAILN=1 step r4s14_step_tile_$r 300 python -u bench.py --no-fft --extra-steps 0 --steps 10 --warmup 3
done
