#!/bin/bash
# Round 4, GPU session 27: execute_v2 latency by binding kind (own buffers, caller pointers copied, caller pointers with a
# bound graph), bench/bench_engine_bindings.py, two processes.
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
python -u -c "import __graft_entry__ as g; g.build()" > gpurun_out/r4s27_build.log 2>&1 || { echo build failed; tail -5 gpurun_out/r4s27_build.log; exit 1; }
TAILN=5 step r4s27_bind_a 300 python -u bench/bench_engine_bindings.py
TAILN=5 step r4s27_bind_b 300 python -u bench/bench_engine_bindings.py
