#!/bin/bash
# Round 4, GPU session 24: LayerNorm fold as two packed FMAs per pair (rstd acc + (bias - rstd mean c1)): GEMM tests, the
# fc1 forms in one process (two processes), and the bench line.
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
python -u -c "import __graft_entry__ as g; g.build()" > gpurun_out/r4s24_build.log 2>&1 || { echo build failed; tail -5 gpurun_out/r4s24_build.log; exit 1; }
TAILN=4 step r4s24_tests 600 python -u -m pytest tests/test_bf16_stats.py tests/test_gemm.py tests/test_fp32_path.py tests/test_spectral_gpu.py tests/test_models.py -x -q -m gpu --timeout 300 --timeout-method thread
TAILN=12 step r4s24_gemm_a 300 python -u bench/bench_gemm.py --rounds 5 && TAILN=12 step r4s24_gemm_b 300 python -u bench/bench_gemm.py --rounds 5
TAILN=1 step r4s24_bench 400 python -u bench.py
