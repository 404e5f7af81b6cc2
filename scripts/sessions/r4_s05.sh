#!/bin/bash
# Round 4, GPU session 5: the fc2 statistics epilogue rewrite (phase clocks, headline step) and the full GPU tier.
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
TAILN=14 step r4s05_gemm_stamps 200 ./variants/bin/gemm_stamps
TAILN=1 step r4s05_bench 400 python -u bench.py --no-fft --extra-steps 0 --steps 10 --warmup 3
TAILN=6 step r4s05_gpu_tier 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider
