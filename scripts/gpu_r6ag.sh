set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
bash $S r6ag_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
bash $S r6ag_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
bash $S r6ag_bench 600 python bench.py --json-out gpurun_out/r6ag_bench.json || exit $?
