#!/bin/bash
# Round 4, GPU session 4: does the operand stream set the MLP GEMMs' power-limited speed?  Same kernels with a
# quarter of the DMA bytes in one (variants/dw2: region R1, -19 % of the L2->LDS bytes) or two (variants/dw6: R1+R2,
# -38 %) of the four regions (-DGEMM_DMA_DWORD, timing only: same instructions and vmcnt counts, wrong values), ABAB.
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
for r in 1 2; do
  TAILN=9 step r4s04_gemm_def_$r 300 python -u bench/bench_gemm.py --x3 --rounds 3
  MI_DFT_LIB=$PWD/variants/dw2/_C.so TAILN=9 step r4s04_gemm_dw2_$r 300 python -u bench/bench_gemm.py --x3 --rounds 3
  MI_DFT_LIB=$PWD/variants/dw6/_C.so TAILN=9 step r4s04_gemm_dw6_$r 300 python -u bench/bench_gemm.py --x3 --rounds 3
done
