#!/bin/bash
# AFNO -O3 corruption, round-3 lead: with the AMDGPU load/store vectorizer ON, afno_spectral.hip is the
# only kernel file whose gfx950 code contains v_swap_b32 (135 of them; 0 with the vectorizer off and 0 in
# gemm / afno_wfft / layernorm / fft / fno kernels, which are all exact with it on).  This builds two
# libraries on the CPU (run here, not on the GPU box):
#   build_diag/vec1/_C.so   afno_spectral.hip with the vectorizer on (the failing configuration)
#   build_diag/vec1x/_C.so  the same device assembly with every `v_swap_b32 a, b` rewritten as the
#                           three-XOR swap (bit-identical semantics, no v_swap_b32 in the code object)
# then scripts/diag/afno_race_diag.py runs against each on the GPU (MI_DFT_LIB=...).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
cd "$ROOT"
VEC="-mllvm -amdgpu-load-store-vectorizer=1"
MI_DFT_HIPCC_EXTRA="$VEC" python -m tensorrt_dft_plugins_amd._build --out build/diag_vec1 -j 8
rm -rf build/diag_vec1x && cp -r build/diag_vec1 build/diag_vec1x
W=$(mktemp -d /tmp/swpXXXX)
SRC=$ROOT/csrc/spectral/afno_spectral.hip
OBJ=$ROOT/build/diag_vec1x/obj/spectral_afno_spectral.hip.o
FLAGS=$(python - <<'EOF'
import sys; sys.path.insert(0, ".")
from tensorrt_dft_plugins_amd import _build
print(f"-D_GLIBCXX_USE_CXX11_ABI={_build._torch_paths()[2]}", " ".join(_build._file_flags("csrc/spectral/afno_spectral.hip")))
EOF
)
# the hipcc pipeline of one .hip file, as commands; run them with the device assembly edited in between
( cd "$W" && /opt/rocm/bin/hipcc -### -c -fPIC -std=c++17 -O3 -I"$ROOT/csrc" \
    -x hip --offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize $FLAGS $VEC -save-temps -o "$OBJ" "$SRC" \
    2>&1 | grep '^ "' > cmds.txt )
DEV_S=afno_spectral-hip-amdgcn-amd-amdhsa-gfx950.s
n=0
while IFS= read -r c; do
  ( cd "$W" && eval "$c" )
  n=$((n + 1))
  if [ -f "$W/$DEV_S" ] && [ ! -f "$W/.edited" ] && echo "$c" | grep -q '"-S"' && echo "$c" | grep -q amdgcn-amd-amdhsa; then
    before=$(grep -c v_swap_b32 "$W/$DEV_S" || true)
    sed -i -E 's/^(\s*)v_swap_b32\s+(v[0-9]+),\s*(v[0-9]+)/\1v_xor_b32 \2, \2, \3\n\1v_xor_b32 \3, \2, \3\n\1v_xor_b32 \2, \2, \3/' "$W/$DEV_S"
    echo "v_swap_b32 in device assembly: $before -> $(grep -c v_swap_b32 "$W/$DEV_S" || true)"
    touch "$W/.edited"
  fi
done < "$W/cmds.txt"
[ -f "$W/.edited" ] || { echo "device assembly step not found"; exit 1; }
touch "$OBJ"
python -m tensorrt_dft_plugins_amd._build --out build/diag_vec1x -j 8
mkdir -p build_diag/vec1 build_diag/vec1x
cp build/diag_vec1/_C.so build_diag/vec1/_C.so
cp build/diag_vec1x/_C.so build_diag/vec1x/_C.so
echo "built build_diag/vec1/_C.so build_diag/vec1x/_C.so ($n pipeline steps)"
