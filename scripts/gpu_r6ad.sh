set -u
S=scripts/gpu_step.sh
bash $S r6ad_tests 600 python -u -m pytest tests/test_fno.py -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
bash $S r6ad_st1 120 ./ab/fno_stamps_tf1 || exit $?
bash $S r6ad_st0 120 ./ab/fno_stamps_tf0 || exit $?
for i in 1 2 3; do
  bash $S r6ad_new_$i 200 python bench/fno_probe.py || exit $?
  MI_DFT_LIB=ab/tf0/_C.so bash $S r6ad_old_$i 200 python bench/fno_probe.py || exit $?
done
