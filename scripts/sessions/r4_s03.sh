#!/bin/bash
# Round 4, GPU session 3: same-box ABAB of the fp32 headline step, this round's code vs the round-3 state
# (variants/r3: git archive of the round-3 final commit, built in-tree) -- the LayerNorm->split pass removed,
# fc1 with LN2 folded, unconditional GEMM epilogue stores -- and the MLP GEMMs (bench_gemm --x3) of both.
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
B="--steps 10 --warmup 3 --no-fft --extra-steps 0"
for r in 1 2; do
  TAILN=1 step r4s03_new_$r 400 python -u bench.py $B
  (cd variants/r3 && TAILN=1 step r4s03_old_$r 400 python -u bench.py $B) || exit 1
done
TAILN=9 step r4s03_gemm_new 300 python -u bench/bench_gemm.py --x3 --rounds 3
(cd variants/r3 && TAILN=6 step r4s03_gemm_old 300 python -u bench/bench_gemm.py --x3 --rounds 3) || exit 1
