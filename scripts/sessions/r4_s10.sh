#!/bin/bash
# Round 4, GPU session 10: bf16 block without LayerNorm-statistics passes (linear_stats + c2r_ln_add_part
# partials merged by ln_stats_merge) -- correctness, then the bf16 and fp32 steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp MI_DFT_BOX_BUILD=0
ROOT=$PWD
step() {
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "$ROOT/gpurun_out/$tag.log" | grep -v "warning: failed to meet" | tail -${TAILN:-12}
  if [ $rc -ne 0 ]; then echo "stopping: $tag failed ($rc)"; exit $rc; fi
}
TAILN=6 step r4s10_tests 500 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread -m gpu tests/test_bf16_stats.py \
  tests/test_spectral_gpu.py tests/test_ln_fused.py tests/test_gemm.py tests/test_gemm_variants.py tests/test_engine.py
TAILN=1 step r4s10_step_1 300 python -u bench.py --no-fft --steps 10 --warmup 3
PROF_TAG=_r4s10b BENCH_ARGS="--dtype bf16" TAILN=14 step r4s10_profb 400 bash scripts/prof_bench.sh
bash scripts/sessions/r4_s12.sh || exit $?
