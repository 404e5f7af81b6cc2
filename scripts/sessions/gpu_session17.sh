#!/bin/bash
# GPU session 18 (round 3): FNO block, batched mixing-gather loads and bf16 dftw on hi-only twiddles (after session 17:
# mixing fused into the inverse H transform, bf16 c2r_pw on hi-only spectra) -- tests, bench, kernel table.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() {
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "gpurun_out/$tag.log" | grep -v "warning: failed to meet" | tail -${TAILN:-12}
  if [ $rc -ne 0 ]; then echo "stopping: $tag failed ($rc)"; exit $rc; fi
}
TAILN=3 step s18_tests 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_fno.py tests/test_dft_gpu.py tests/test_determinism_gpu.py
TAILN=3 step s18_fno 300 python -u bench/bench_fno.py --amd-only --rounds 10
TAILN=3 step s18_fno2 300 python -u bench/bench_fno.py --amd-only --rounds 10
step s18_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fno18 -o fno -- python3 bench/bench_fno.py --amd-only --rounds 3
python3 scripts/kernel_summary.py gpurun_out/prof_fno18 | head -12
