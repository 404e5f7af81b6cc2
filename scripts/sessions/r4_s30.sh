#!/bin/bash
# Round 4, GPU session 30 (final commit of the round): the tier as the driver runs it (library compiled from source on the
# box by the tier's conftest), smoke(), the full bench line, and a kernel table of the fp32 headline.
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
TAILN=5 step r4s30_tier 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
TAILN=2 step r4s30_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
TAILN=1 step r4s30_bench 400 python -u bench.py
