#!/bin/bash
# One GPU session (round 3): correctness tiers for the changed kernel families, then the GEMM DMA
# placement A/B, the FFT latency and the headline bench.  Every GPU step has its own time limit;
# the session stops at the first abnormal exit (timeout, signal, fault).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # step <tag> <seconds> <cmd...>
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "gpurun_out/$tag.log" | tail -${TAILN:-6}
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $tag ended abnormally ($rc)"; exit $rc; fi
  return $rc
}
step s_build_mid0 600 env MI_DFT_HIPCC_EXTRA="-DGEMM_DMA_MID=0" python -u -m tensorrt_dft_plugins_amd._build --force --out build/mid0 -j 16 || exit 1
step s_tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gemm.py tests/test_fp32_path.py \
  tests/test_ln_fused.py tests/test_patch_gemm.py tests/test_dft_gpu.py tests/test_fno.py tests/test_spectral_gpu.py tests/test_engine.py
TAILN=30 step s_fft 300 python -u bench/bench_fft.py --rounds 10
for r in 1 2; do
  TAILN=5 step s_gemm_mid1_$r 300 python -u bench/bench_gemm.py --x3 --rounds 3
  TAILN=5 step s_gemm_mid0_$r 300 env MI_DFT_LIB=$PWD/build/mid0/_C.so python -u bench/bench_gemm.py --x3 --rounds 3
done
TAILN=3 step s_bench 500 python -u bench.py --steps 10 --warmup 3
