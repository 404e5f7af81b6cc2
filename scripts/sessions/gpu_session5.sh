#!/bin/bash
# GPU session 5 (round 3): AFNO x3 phase clocks and the transposed-GEMM1 epilogue A/B, then the
# from-source CI (compile on the box + both tiers).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for t in 1 0; do
  timeout -k 10 300 hipcc -O3 -mllvm -amdgpu-load-store-vectorizer=0 --offload-arch=gfx950 -munsafe-fp-atomics \
    -fno-slp-vectorize -DAFNO_STAMPS -DAFNO_X3_T=$t -Icsrc bench/afno_stamps.hip -o /tmp/afno_stamps$t || exit 1
  timeout -k 10 120 /tmp/afno_stamps$t > gpurun_out/s5_afno_stamps_t$t.log 2>&1; rc=$?
  echo "== AFNO_X3_T=$t"; cat gpurun_out/s5_afno_stamps_t$t.log
  [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  timeout -k 10 200 python -u bench/bench_afno_spec.py > gpurun_out/s5_spec_t1_$r.log 2>&1 || exit $?
  echo "T=1: $(tail -1 gpurun_out/s5_spec_t1_$r.log)"
  MI_DFT_LIB=$PWD/build_diag/x3t0/_C.so timeout -k 10 200 python -u bench/bench_afno_spec.py > gpurun_out/s5_spec_t0_$r.log 2>&1 || exit $?
  echo "T=0: $(tail -1 gpurun_out/s5_spec_t0_$r.log)"
done
bash scripts/ci_gpu.sh 2>&1 | tee gpurun_out/s5_ci.log
