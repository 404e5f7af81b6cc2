#!/bin/bash
# Round 4, GPU session 21: the cost of the bf16 fc2 statistics epilogue in one process (fc2 + residual with and
# without the next LayerNorm's partials, bench/bench_gemm.py, two processes).
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
python -u -c "import __graft_entry__ as g; g.build()" > gpurun_out/r4s21_build.log 2>&1 || { echo build failed; tail -5 gpurun_out/r4s21_build.log; exit 1; }
TAILN=12 step r4s21_gemm_a 300 python -u bench/bench_gemm.py --rounds 5
TAILN=12 step r4s21_gemm_b 300 python -u bench/bench_gemm.py --rounds 5
