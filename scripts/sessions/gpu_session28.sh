#!/bin/bash
# GPU session 28 (round 3, end of the re-entry session): from-source CI on the box (scripts/ci_gpu.sh: build every
# source into build/box, CPU tier + GPU tier against it), then smoke() and bench.py on the in-tree library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1100 bash scripts/ci_gpu.sh > gpurun_out/s28_ci.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/s28_ci.log | tail -12
[ $rc -eq 0 ] || { echo "ci ended with $rc"; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s28_smoke.log 2>&1 || { tail -5 gpurun_out/s28_smoke.log; exit 1; }
tail -1 gpurun_out/s28_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/s28_bench.log 2>&1 || { tail -5 gpurun_out/s28_bench.log; exit 1; }
tail -1 gpurun_out/s28_bench.log
