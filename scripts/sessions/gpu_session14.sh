#!/bin/bash
# GPU session 14 (round 3, re-entry): full GPU tier + smoke + bench on the in-tree build, and the FNO block bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "gpurun_out/$tag.log" | grep -v "warning: failed to meet" | tail -${TAILN:-12}
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $tag ended abnormally ($rc)"; exit $rc; fi
  return $rc
}
TAILN=4 step s14_tests 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests
TAILN=2 step s14_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
TAILN=3 step s14_bench 600 python -u bench.py
TAILN=3 step s14_fno 300 python -u bench/bench_fno.py --amd-only --rounds 10
