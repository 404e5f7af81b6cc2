set -u
S=scripts/gpu_step.sh
bash $S r6a_tests 900 python -u -m pytest tests/test_dp.py tests/test_optimizer_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
bash $S r6a_bench 600 python bench.py --json-out gpurun_out/r6a_bench.json || exit $?
