#!/bin/bash
# Round 4, GPU session 1: the fp32 block without the LayerNorm->split pass (c2r_ln_add_split + linear3_ln) --
# its GPU tests (library compiled from source on the box by the GPU-tier conftest), the headline bench and a
# per-kernel table; the persistent fp32-block GEMMs (bit-exact test, GEMM and bench A/B). (FNO mixing paths: session 2.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "gpurun_out/$tag.log" | grep -v "warning: failed to meet" | tail -${TAILN:-12}
  if [ $rc -ne 0 ]; then echo "stopping: $tag failed ($rc)"; exit $rc; fi
}
TAILN=6 step r4s01_tests 700 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread -m gpu tests/test_fp32_path.py tests/test_fno.py -k "ln or split or full_depth or fp32_amd or mix"
TAILN=4 step r4s01_persist_test 400 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu tests/test_gemm_variants.py -k persistent
TAILN=3 step r4s01_bench 400 python -u bench.py
TAILN=8 step r4s01_gemm_p0 300 env MI_DFT_GEMM_PERSIST=0 python -u bench/bench_gemm.py --x3 --rounds 3
TAILN=8 step r4s01_gemm_p1 300 env MI_DFT_GEMM_PERSIST=1 python -u bench/bench_gemm.py --x3 --rounds 3
TAILN=3 step r4s01_bench_p1 400 env MI_DFT_GEMM_PERSIST=1 python -u bench.py
PROF_TAG=_r4s01 timeout -k 10 700 bash scripts/prof_bench.sh > gpurun_out/r4s01_prof.txt 2>&1; echo "prof rc=$?"; head -16 gpurun_out/r4s01_prof.txt
python3 scripts/trace_window.py gpurun_out/prof_bench_r4s01 > gpurun_out/r4s01_window.txt 2>&1; head -30 gpurun_out/r4s01_window.txt
