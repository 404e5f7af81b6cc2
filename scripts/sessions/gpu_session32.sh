#!/bin/bash
# GPU session 32 (round 3, final): afno_spectral.hip back on the default flags (vectorizer on) now that radix.h's c_mul
# no longer produces the faulting packed-FP32 form -- AFNO race screen x2, H-filter speed, full GPU tier, smoke, bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/diag/afno_race_diag.py > gpurun_out/s32_afno_$rep.log 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/s32_afno_$rep.log | tail -5; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u bench/bench_afno_spec.py > gpurun_out/s32_spec_$rep.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/s32_spec_$rep.log | tail -1
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/s32_tests.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/s32_tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s32_smoke.log 2>&1 || { tail -5 gpurun_out/s32_smoke.log; exit 1; }
tail -1 gpurun_out/s32_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/s32_bench.log 2>&1 || { tail -5 gpurun_out/s32_bench.log; exit 1; }
tail -1 gpurun_out/s32_bench.log
