set -u
S=scripts/gpu_step.sh
export MI_DFT_LIB=ab/tune/_C.so
for i in 1 2; do
  bash $S r6s_def_$i 200 python bench/fno_probe.py || exit $?
  for c in 90,2 90,8 45,4 45,8; do
    MI_DFT_FIXED_CFG=$c bash $S r6s_c${c/,/_}_$i 200 python bench/fno_probe.py || exit $?
  done
done
