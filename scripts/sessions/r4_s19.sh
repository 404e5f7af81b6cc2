#!/bin/bash
# Round 4, GPU session 19: bf16 AFNO C2R partials written over the lane's own residual slot (one barrier fewer);
# tests, the bf16 kernel table and steps.
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
TAILN=3 step r4s19_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_bf16_stats.py \
  tests/test_ln_fused.py tests/test_spectral_gpu.py tests/test_patch_gemm.py
PROF_TAG=_r4s19b BENCH_ARGS="--dtype bf16" TAILN=10 step r4s19_profb 400 bash scripts/prof_bench.sh
TAILN=1 step r4s19_bench 400 python -u bench.py --no-fft --steps 10 --warmup 3
