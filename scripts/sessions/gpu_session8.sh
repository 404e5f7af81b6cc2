#!/bin/bash
# GPU session 8 (round 3): persistent AFNO x3 kernel with the next tile's input DMA'd into LDS.
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
TAILN=6 step s8_tests 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_spectral_gpu.py tests/test_fp32_path.py tests/test_determinism_gpu.py
step s8_build_stamps 300 hipcc -O3 -mllvm -amdgpu-load-store-vectorizer=0 --offload-arch=gfx950 -munsafe-fp-atomics \
  -fno-slp-vectorize -DAFNO_STAMPS -Icsrc bench/afno_stamps.hip -o /tmp/afno_stamps || exit 1
TAILN=14 step s8_afno_stamps 120 /tmp/afno_stamps
TAILN=2 step s8_spec1 200 python -u bench/bench_afno_spec.py
TAILN=2 step s8_spec1_np 200 env MI_DFT_AFNO_PERSIST=0 python -u bench/bench_afno_spec.py
TAILN=2 step s8_spec2 200 python -u bench/bench_afno_spec.py
TAILN=2 step s8_spec2_np 200 env MI_DFT_AFNO_PERSIST=0 python -u bench/bench_afno_spec.py
TAILN=2 step s8_bench 600 python -u bench.py --steps 10 --warmup 3
TAILN=2 step s8_bench_np 600 env MI_DFT_AFNO_PERSIST=0 python -u bench.py --steps 10 --warmup 3 --no-fft --extra-steps 0
