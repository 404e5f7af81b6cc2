#!/bin/bash
# GPU session 30 (round 3, final state of the re-entry session): full GPU tier, smoke(), bench.py on the in-tree library
# (what the driver runs at round end), and the bf16 FNO block.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/s30_tests.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/s30_tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s30_smoke.log 2>&1 || { tail -5 gpurun_out/s30_smoke.log; exit 1; }
tail -1 gpurun_out/s30_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/s30_bench.log 2>&1 || { tail -5 gpurun_out/s30_bench.log; exit 1; }
tail -1 gpurun_out/s30_bench.log
