#!/bin/bash
# GPU session 2 (round 3): in-step marginal cost of every fp32 block stage (no profiler), the
# AFNO -O3 bisection, and the FFT after the column-layout change.
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
step s2_fft_tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_dft_gpu.py tests/test_fno.py
TAILN=12 step s2_fft 300 python -u bench/bench_fft.py --rounds 10
TAILN=12 step s2_marginal 900 python -u bench/marginal_cost.py --steps 6
TAILN=40 step s2_afno_bisect 900 bash scripts/diag/afno_o3_bisect.sh
