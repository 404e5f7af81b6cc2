#!/bin/bash
# GPU session 10 (round 3): full GPU tier, smoke, headline bench, kernel table of the final state.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "gpurun_out/$tag.log" | tail -${TAILN:-12}
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $tag ended abnormally ($rc)"; exit $rc; fi
  return $rc
}
TAILN=3 step s10_tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests
TAILN=2 step s10_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
TAILN=2 step s10_bench 600 python -u bench.py --steps 10 --warmup 3
TAILN=2 step s10_bench2 600 python -u bench.py --steps 10 --warmup 3
TAILN=30 PROF_TAG=_r3b step s10_prof 700 bash scripts/prof_bench.sh
