#!/bin/bash
# GPU session 12 (round 3): FNO layer tail phase clocks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize -DFNO_STAMPS -Icsrc \
  bench/fno_stamps.hip -o /tmp/fno_stamps || exit 1
timeout -k 10 120 /tmp/fno_stamps > gpurun_out/s12_fno_stamps.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/s12_fno_stamps.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_fno.py > gpurun_out/s12_tests.log 2>&1; rc=$?
tail -2 gpurun_out/s12_tests.log
exit $rc
