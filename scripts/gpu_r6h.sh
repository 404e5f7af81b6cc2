set -u
S=scripts/gpu_step.sh
bash $S r6h_tests 900 python -u -m pytest tests/test_gemm.py tests/test_gemm_ragged.py tests/test_fp32_path.py tests/test_patch_gemm.py tests/test_determinism_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
for i in 1 2; do
  bash $S r6h_stamps_new_$i 300 ./stampbin/gemm_stamps || exit $?
  bash $S r6h_stamps_old_$i 300 ./stampbin/gemm_stamps_bal0 || exit $?
done
for i in 1 2; do
  bash $S r6h_gemm_new_$i 400 python bench/bench_gemm.py --x3 --rounds 3 || exit $?
  MI_DFT_LIB=ab/bal0_C.so bash $S r6h_gemm_old_$i 400 python bench/bench_gemm.py --x3 --rounds 3 || exit $?
done
bash $S r6h_bench_new 600 python bench.py --no-fft --native-steps 0 --json-out gpurun_out/r6h_bench_new.json || exit $?
MI_DFT_LIB=ab/bal0_C.so MI_DFT_BENCH_BUILD=0 bash $S r6h_bench_old 600 python bench.py --no-fft --native-steps 0 --json-out gpurun_out/r6h_bench_old.json || exit $?
