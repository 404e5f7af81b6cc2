#!/bin/bash
# Round 4, GPU session 23: where the bf16 fc2 statistics epilogue spends its +80 us -- timing-only builds
# (GEMM_STATS_ABL: 1 no sweep, 2 no partials store, 7 neither nor the staging write-back), bench_gemm per library.
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
python -u -c "import __graft_entry__ as g; g.build()" > gpurun_out/r4s23_build.log 2>&1 || { echo build failed; tail -5 gpurun_out/r4s23_build.log; exit 1; }
TAILN=4 step r4s23_gemm_def 300 python -u bench/bench_gemm.py --rounds 5
for v in 1 2 7; do MI_DFT_LIB=$ROOT/variants/sabl$v/_C.so TAILN=4 step r4s23_gemm_sabl$v 300 python -u bench/bench_gemm.py --rounds 5; done
TAILN=4 step r4s23_gemm_def2 300 python -u bench/bench_gemm.py --rounds 5
