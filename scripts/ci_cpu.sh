#!/bin/bash
# CPU-box CI (no GPU needed; hipcc cross-compiles gfx950):
#   1. CMake + Ninja build of _C.so (CMakeLists.txt) into build/cmake/lib, and the CPU test tier
#      against it (MI_DFT_LIB);
#   2. setup.py build_ext --inplace (the pip-install build path, setup.py -> _build.py);
#   3. host AddressSanitizer build (build/asan/_C.so) and the CPU test tier under ASan.
# Reference: the CMake / setup.py pair of /root/reference/src/dft_plugins/CMakeLists.txt:22-43,
# /root/reference/setup.py:30-48 (built there, never tested).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
step() { echo "== $1"; }
step "cmake build"
cmake -S . -B build/cmake -G Ninja -DMI_DFT_OUTPUT_DIR="$PWD/build/cmake/lib" > gpurun_out/ci_cmake.log 2>&1 &&
  cmake --build build/cmake -j 8 >> gpurun_out/ci_cmake.log 2>&1 || { tail -30 gpurun_out/ci_cmake.log; exit 1; }
step "cpu tier on the CMake-built library"
MI_DFT_LIB="$PWD/build/cmake/lib/_C.so" timeout -k 10 1200 python -m pytest tests -q -x -m "not gpu" -p no:cacheprovider \
  > gpurun_out/ci_cmake_tests.log 2>&1 || { tail -30 gpurun_out/ci_cmake_tests.log; exit 1; }
tail -1 gpurun_out/ci_cmake_tests.log
step "setup.py build_ext --inplace"
timeout -k 10 1200 python setup.py build_ext --inplace > gpurun_out/ci_setup.log 2>&1 || { tail -30 gpurun_out/ci_setup.log; exit 1; }
python -c "import tensorrt_dft_plugins_amd as t; t.load_plugins(); assert {'Rfft','Irfft'} <= t.plugin_names(); print('setup.py build loads:', t.native_library_path())"
step "host ASan build + cpu tier"
python -m tensorrt_dft_plugins_amd._build --asan > gpurun_out/ci_asan_build.log 2>&1 || { tail -30 gpurun_out/ci_asan_build.log; exit 1; }
ASAN_RT=$(ls /opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
LD_PRELOAD="$ASAN_RT" ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0 MI_DFT_LIB="$PWD/build/asan/_C.so" \
  timeout -k 10 1800 python -m pytest tests -q -x -m "not gpu" -p no:cacheprovider > gpurun_out/ci_asan_tests.log 2>&1 \
  || { tail -40 gpurun_out/ci_asan_tests.log; exit 1; }
tail -1 gpurun_out/ci_asan_tests.log
echo "ci_cpu: all green"
