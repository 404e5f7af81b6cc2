#!/bin/bash
# AFNO -O3 corruption bisection on the GPU box: build csrc/ with the load/store vectorizer ON for
# the AFNO spectral file (the failing configuration), with and without the AFNO_DIAG wait-state
# guards, each into its own directory, and run the error / determinism screen on each library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in "vec1:" "vec1_d1:-DAFNO_DIAG=1" "vec1_d2:-DAFNO_DIAG=2" "vec0:"; do
  tag=${v%%:*}; extra=${v#*:}
  vec="-mllvm -amdgpu-load-store-vectorizer=1"; [ "$tag" = vec0 ] && vec=""
  MI_DFT_HIPCC_EXTRA="$vec $extra" timeout -k 10 600 python -u -m tensorrt_dft_plugins_amd._build --force --out build/diag_$tag -j 16 \
    > gpurun_out/afno_bisect_build_$tag.log 2>&1 || { echo "build $tag failed"; tail -5 gpurun_out/afno_bisect_build_$tag.log; exit 1; }
  echo "== $tag ($vec $extra)"
  MI_DFT_LIB=$PWD/build/diag_$tag/_C.so timeout -k 10 300 python -u scripts/diag/afno_race_diag.py 2>&1 | grep -v amdgpu.ids \
    || { echo "diag $tag ended abnormally"; exit 1; }
done
