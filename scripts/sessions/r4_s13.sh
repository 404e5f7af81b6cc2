#!/bin/bash
# Round 4, GPU session 13: single-sweep shifted LN partials (GEMM fc2 epilogue, AFNO C2R fp32 / bf16 epilogues);
# bf16 AFNO spectral kernel at 4 workgroups per CU (variants/occ4) vs 3, ABAB on the bf16 step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp MI_DFT_BOX_BUILD=0
ROOT=$PWD
OCC4=$PWD/variants/occ4/_C.so
step() {
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "$ROOT/gpurun_out/$tag.log" | grep -v "warning: failed to meet" | tail -${TAILN:-12}
  if [ $rc -ne 0 ]; then echo "stopping: $tag failed ($rc)"; exit $rc; fi
}
TAILN=4 step r4s13_tests 500 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread -m gpu tests/test_bf16_stats.py \
  tests/test_fp32_path.py tests/test_ln_fused.py tests/test_gemm_variants.py
MI_DFT_LIB=$OCC4 TAILN=3 step r4s13_tests_occ4 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_spectral_gpu.py
for r in 1 2; do
  TAILN=1 step r4s13_bf16_def_$r 300 python -u bench.py --no-fft --dtype bf16 --extra-steps 0 --steps 10 --warmup 3
  MI_DFT_LIB=$OCC4 TAILN=1 step r4s13_bf16_occ4_$r 300 python -u bench.py --no-fft --dtype bf16 --extra-steps 0 --steps 10 --warmup 3
done
TAILN=1 step r4s13_fp32 300 python -u bench.py --no-fft --extra-steps 0 --steps 10 --warmup 3
PROF_TAG=_r4s13b BENCH_ARGS="--dtype bf16" TAILN=14 step r4s13_profb 400 bash scripts/prof_bench.sh
