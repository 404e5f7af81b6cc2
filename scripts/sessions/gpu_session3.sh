#!/bin/bash
# GPU session 3 (round 3): FNO staged-epilogue A/B, AFNO vectorizer-on build with device LDS checks,
# GEMM per-call time under sustained load, IPC push interference.
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
step s3_build_epi0 600 env MI_DFT_HIPCC_EXTRA="-DFNO_EPI_STAGED=0" python -u -m tensorrt_dft_plugins_amd._build --force --out build/epi0 -j 16 || exit 1
step s3_build_chk 600 env MI_DFT_DEVICE_CHECKS=1 MI_DFT_HIPCC_EXTRA="-mllvm -amdgpu-load-store-vectorizer=1" python -u -m tensorrt_dft_plugins_amd._build --force --out build/chk -j 16 || exit 1
step s3_fno_tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_fno.py tests/test_determinism_gpu.py
for r in 1 2; do
  TAILN=4 step s3_fno_staged_$r 300 python -u bench/bench_fno.py --amd-only --rounds 10
  TAILN=4 step s3_fno_direct_$r 300 env MI_DFT_LIB=$PWD/build/epi0/_C.so python -u bench/bench_fno.py --amd-only --rounds 10
done
TAILN=14 step s3_afno_chk 300 env MI_DFT_LIB=$PWD/build/chk/_C.so python -u scripts/diag/afno_race_diag.py
TAILN=6 step s3_gemm_iters30 300 python -u bench/bench_gemm.py --x3 --rounds 3 --iters 30
TAILN=6 step s3_push 600 python -u bench/push_interference.py --dtype fp32 --ndst 1,3 --steps 6
