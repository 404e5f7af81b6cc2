set -u
S=scripts/gpu_step.sh
for i in 1 2 3 4; do
  bash $S r6af_p0_$i 400 python bench.py --no-fft --native-steps 0 --extra-steps 10 --steps 30 --warmup 5 || exit $?
  MI_DFT_LIB=ab/p2/_C.so bash $S r6af_p2_$i 400 python bench.py --no-fft --native-steps 0 --extra-steps 10 --steps 30 --warmup 5 || exit $?
done
