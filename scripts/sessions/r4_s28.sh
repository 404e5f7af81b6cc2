#!/bin/bash
# Round 4, GPU session 28: execute_v2 hot path for an already bound pointer set (no wrappers or checks): engine GPU tests and
# the binding-kind latency bench.
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
python -u -c "import __graft_entry__ as g; g.build()" > gpurun_out/r4s28_build.log 2>&1 || { echo build failed; tail -5 gpurun_out/r4s28_build.log; exit 1; }
TAILN=4 step r4s28_engine 300 python -u -m pytest tests/test_engine.py -x -q -s -m gpu --timeout 200 --timeout-method thread
TAILN=5 step r4s28_bind_a 300 python -u bench/bench_engine_bindings.py
TAILN=5 step r4s28_bind_b 300 python -u bench/bench_engine_bindings.py
