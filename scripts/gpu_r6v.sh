set -u
S=scripts/gpu_step.sh
bash $S r6v_tests 600 python -u -m pytest tests/test_fno.py tests/test_optimizer_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
bash $S r6v_st_new 120 ./ab/fno_stamps_new || exit $?
bash $S r6v_st_old 120 ./ab/fno_stamps_old || exit $?
for i in 1 2 3; do
  bash $S r6v_new_$i 200 python bench/fno_probe.py || exit $?
  MI_DFT_LIB=ab/old/_C.so bash $S r6v_old_$i 200 python bench/fno_probe.py || exit $?
done
