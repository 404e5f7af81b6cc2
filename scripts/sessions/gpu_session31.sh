#!/bin/bash
# GPU session 31 (round 3): the fix at the source (radix.h c_mul(cpair, float2): the twiddle's imaginary part through its
# own register, so no packed-FP32 op takes src1's high half via op_sel -- 0 such instructions in all 893 kernels).
# (1) causal check: the AFNO race screen on a vectorizer-ON build with the fix (diag_libs/vecfix) and on the shipped
# (vectorizer-off) build with the fix; (2) AFNO H-filter speed, both builds; (3) full GPU tier, smoke, bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2; do
  for t in vecfix shipped; do
    lib=$PWD/diag_libs/$t/_C.so; [ $t = shipped ] && lib=$PWD/tensorrt_dft_plugins_amd/_C.so
    echo "== afno $t rep $rep"
    MI_DFT_LIB=$lib timeout -k 10 300 python -u scripts/diag/afno_race_diag.py > gpurun_out/s31_afno_${t}_$rep.log 2>&1; rc=$?
    grep -v amdgpu.ids gpurun_out/s31_afno_${t}_$rep.log | tail -3; [ $rc -eq 0 ] || { echo "afno $t ended abnormally ($rc)"; exit $rc; }
    MI_DFT_LIB=$lib timeout -k 10 300 python -u bench/bench_afno_spec.py > gpurun_out/s31_spec_${t}_$rep.log 2>&1 || { echo "spec bench $t failed"; exit 1; }
    grep -v amdgpu.ids gpurun_out/s31_spec_${t}_$rep.log | tail -2
  done
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/s31_tests.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/s31_tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s31_smoke.log 2>&1 || { tail -5 gpurun_out/s31_smoke.log; exit 1; }
tail -1 gpurun_out/s31_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/s31_bench.log 2>&1 || { tail -5 gpurun_out/s31_bench.log; exit 1; }
tail -1 gpurun_out/s31_bench.log
