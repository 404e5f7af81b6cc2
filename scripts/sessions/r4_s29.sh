#!/bin/bash
# Round 4, GPU session 29: kernel table of the bf16 FourCastNet step on the final tree (rocprofv3 --kernel-trace --stats).
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
python -u -c "import __graft_entry__ as g; g.build()" > gpurun_out/r4s29_build.log 2>&1 || { echo build failed; tail -5 gpurun_out/r4s29_build.log; exit 1; }
PROF_TAG=_r4final_bf16 BENCH_ARGS="--dtype bf16" TAILN=16 step r4s29_prof 500 bash scripts/prof_bench.sh
