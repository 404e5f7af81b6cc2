set -u
S=scripts/gpu_step.sh
bash $S r6y_tests 600 python -u -m pytest tests/test_fno.py tests/test_optimizer_gpu.py tests/test_dft_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
bash $S r6y_rows_new 200 python bench/dftw_rows.py || exit $?
MI_DFT_LIB=ab/nobal/_C.so bash $S r6y_rows_old 200 python bench/dftw_rows.py || exit $?
for i in 1 2 3; do
  bash $S r6y_new_$i 200 python bench/fno_probe.py || exit $?
  MI_DFT_LIB=ab/nobal/_C.so bash $S r6y_old_$i 200 python bench/fno_probe.py || exit $?
done
