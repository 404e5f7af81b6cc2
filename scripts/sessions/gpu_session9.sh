#!/bin/bash
# GPU session 9 (round 3): what limits the bf16 GEMM main loop -- phase clocks with the main-loop DMA removed
# (GEMM_ABLATE=1), the fragment reads removed (2), both (3); timing-only builds, results are wrong.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for a in 0 1 2 3; do
  timeout -k 10 300 hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize -DAMD_DFT_GEMM_STAMPS \
    -DGEMM_ABLATE=$a -Icsrc bench/gemm_stamps.hip -o /tmp/gst$a || exit 1
  echo "== GEMM_ABLATE=$a"
  timeout -k 10 200 /tmp/gst$a > gpurun_out/s9_gst$a.log 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/s9_gst$a.log
  [ $rc -eq 0 ] || exit $rc
done
