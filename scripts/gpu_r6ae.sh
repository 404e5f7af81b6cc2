set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
bash $S r6ae_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
bash $S r6ae_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
