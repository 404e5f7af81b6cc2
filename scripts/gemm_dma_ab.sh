#!/bin/bash
# A/B of the GEMM DMA placement (GEMM_DMA_MID=1, in-tree default, vs 0) on the GPU box:
# correctness of the in-tree build first (GEMM + fp32-path GPU tests), then bench/bench_gemm.py
# --x3 per build, ABAB (two libraries cannot share one process: same op names).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
MI_DFT_HIPCC_EXTRA="-DGEMM_DMA_MID=0" timeout -k 10 600 python -u -m tensorrt_dft_plugins_amd._build --force --out build/mid0 -j 16 \
  > gpurun_out/gemm_ab_build.log 2>&1 || { tail -5 gpurun_out/gemm_ab_build.log; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm.py tests/test_fp32_path.py \
  tests/test_ln_fused.py tests/test_patch_gemm.py -m gpu > gpurun_out/gemm_ab_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gemm_ab_tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in mid1 mid0; do
    lib=""; [ $v = mid0 ] && lib="$PWD/build/mid0/_C.so"
    echo "== $v round $r"
    MI_DFT_LIB=$lib timeout -k 10 300 python -u bench/bench_gemm.py --x3 --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
