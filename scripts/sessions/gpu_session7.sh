#!/bin/bash
# GPU session 7 (round 3): last block's fc2 writing the head operand as split pairs; x3 GEMM bench with full
# fp32 operands (non-zero lo halves) vs the old zero-lo harness.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "gpurun_out/$tag.log" | tail -${TAILN:-12}
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $tag ended abnormally ($rc)"; exit $rc; fi
  return $rc
}
TAILN=4 step s7_tests 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_fp32_path.py tests/test_engine.py
TAILN=2 step s7_bench 600 python -u bench.py --steps 10 --warmup 3
TAILN=2 step s7_bench_nohead 600 env MI_DFT_HEAD_SPLIT=0 python -u bench.py --steps 10 --warmup 3
TAILN=6 step s7_gemm_full 400 python -u bench/bench_gemm.py --x3 --rounds 3
TAILN=6 step s7_gemm_zerolo 400 python -u bench/bench_gemm.py --x3 --rounds 3 --zero-lo
