set -u
S=scripts/gpu_step.sh
for i in 1 2; do
  for mo in one seq2 mb2; do
    bash $S r6l_${mo}_$i 240 python bench/bench_mbatch.py --mode $mo || exit $?
  done
done
