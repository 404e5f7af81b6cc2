set -u
S=scripts/gpu_step.sh
bash $S r6ac_tests 600 python -u -m pytest tests/test_fno.py -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
