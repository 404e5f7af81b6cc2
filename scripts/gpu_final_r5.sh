set -u
S=scripts/gpu_step.sh
bash $S r5h_tests 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
bash $S r5h_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
bash $S r5h_bench 600 python bench.py || exit $?
