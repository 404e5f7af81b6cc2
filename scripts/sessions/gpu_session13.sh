#!/bin/bash
# GPU session 13 (round 3): FNO kernels with their first loads issued before the table setup -- tests, phase
# clocks, and the FNO block A/B/C: + lane-transposed 16-byte bf16 stores (in-tree), without them
# (build_diag/fnonoswap), the previous build (build_diag/fnoprev).
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
TAILN=3 step s13_tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_fno.py tests/test_dft_gpu.py
step s13_build_stamps 300 hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize -DFNO_STAMPS -Icsrc \
  bench/fno_stamps.hip -o /tmp/fno_stamps || exit 1
TAILN=16 step s13_fno_stamps 120 /tmp/fno_stamps
for r in 1 2; do
  TAILN=3 step s13_fno_new_$r 300 python -u bench/bench_fno.py --amd-only --rounds 10
  TAILN=3 step s13_fno_noswap_$r 300 env MI_DFT_LIB=$PWD/build_diag/fnonoswap/_C.so python -u bench/bench_fno.py --amd-only --rounds 10
  TAILN=3 step s13_fno_prev_$r 300 env MI_DFT_LIB=$PWD/build_diag/fnoprev/_C.so python -u bench/bench_fno.py --amd-only --rounds 10
done
TAILN=30 step s13_kernels 300 python -u bench/bench_kernels_fno.py
