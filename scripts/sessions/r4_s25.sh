#!/bin/bash
# Round 4, GPU session 25 (final tree of the round): the GPU tier as the driver runs it (library compiled from source on the
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
TAILN=5 step r4s25_tier 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
TAILN=2 step r4s25_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
TAILN=1 step r4s25_bench 400 python -u bench.py
PROF_TAG=_r4final3 TAILN=14 step r4s25_prof 400 bash scripts/prof_bench.sh
