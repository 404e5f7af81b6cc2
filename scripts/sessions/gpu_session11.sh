#!/bin/bash
# GPU session 11 (round 3): bf16 AFNO kernel with the transposed GEMM-1 epilogue.
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
TAILN=3 step s11_tests 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_spectral_gpu.py tests/test_determinism_gpu.py tests/test_fp32_path.py tests/test_models.py
TAILN=6 step s11_race 200 python -u scripts/diag/afno_race_diag.py
TAILN=2 step s11_spec1 200 python -u bench/bench_afno_spec.py
TAILN=2 step s11_spec2 200 python -u bench/bench_afno_spec.py
