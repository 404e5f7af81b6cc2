#!/bin/bash
# Round 4, GPU session 8: the two-phase GEMM default -- full GPU tier, smoke, the full bench line, and
# rocprofv3 kernel tables of the fp32 headline and the bf16 model.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp MI_DFT_BOX_BUILD=0
ROOT=$PWD
step() {
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "$ROOT/gpurun_out/$tag.log" | grep -v "warning: failed to meet" | tail -${TAILN:-12}
  if [ $rc -ne 0 ]; then echo "stopping: $tag failed ($rc)"; exit $rc; fi
}
TAILN=4 step r4s08_tier 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
TAILN=2 step r4s08_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
TAILN=1 step r4s08_bench 400 python -u bench.py
PROF_TAG=_r4h TAILN=16 step r4s08_prof 400 bash scripts/prof_bench.sh
PROF_TAG=_r4hb BENCH_ARGS="--dtype bf16" TAILN=16 step r4s08_profb 400 bash scripts/prof_bench.sh
