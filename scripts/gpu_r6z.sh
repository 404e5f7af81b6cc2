set -u
S=scripts/gpu_step.sh
for i in 1 2; do
  bash $S r6z_gemm_p0_$i 300 python bench/bench_gemm.py --x3 --rounds 3 || exit $?
  MI_DFT_LIB=ab/p1/_C.so bash $S r6z_gemm_p1_$i 300 python bench/bench_gemm.py --x3 --rounds 3 || exit $?
  MI_DFT_LIB=ab/p2/_C.so bash $S r6z_gemm_p2_$i 300 python bench/bench_gemm.py --x3 --rounds 3 || exit $?
done
