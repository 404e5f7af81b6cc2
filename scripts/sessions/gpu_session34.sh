#!/bin/bash
# GPU session 34 (round 3, last): GPU tier + smoke on the in-tree library as rebuilt by setup.py (scripts/ci_cpu.sh), then
# the FNO column-tile A/B of session 33 (which never got a box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/s34_tests.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/s34_tests.log | tail -1; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s34_smoke.log 2>&1 || { tail -5 gpurun_out/s34_smoke.log; exit 1; }
tail -1 gpurun_out/s34_smoke.log
bash scripts/sessions/gpu_session33.sh
