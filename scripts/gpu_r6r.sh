set -u
S=scripts/gpu_step.sh
bash $S r6r_tests 600 python -u -m pytest tests/test_fno.py tests/test_optimizer_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
for i in 1 2 3; do
  bash $S r6r_probe_$i 200 python bench/fno_probe.py || exit $?
done
