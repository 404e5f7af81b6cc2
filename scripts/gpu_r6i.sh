set -u
S=scripts/gpu_step.sh
bash $S r6i_tests 900 python -u -m pytest tests/test_fno.py tests/test_optimizer_gpu.py -m gpu -x -q --timeout 600 --timeout-method thread || exit $?
for i in 1 2; do
  bash $S r6i_fno_new_$i 200 python bench/bench_fno.py --amd-only --rounds 10 || exit $?
  MI_DFT_LIB=ab/actsc_C.so bash $S r6i_fno_sc_$i 200 python bench/bench_fno.py --amd-only --rounds 10 || exit $?
  MI_DFT_LIB=ab/acttanh_C.so bash $S r6i_fno_tanh_$i 200 python bench/bench_fno.py --amd-only --rounds 10 || exit $?
done
