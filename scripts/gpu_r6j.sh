set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
bash $S r6j_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
bash $S r6j_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
bash $S r6j_bench 600 python bench.py --json-out gpurun_out/r6j_bench.json || exit $?
PROF_TAG=_r6j_fp32 BENCH_ARGS="--native-steps 0" bash scripts/prof_bench.sh > gpurun_out/r6j_prof_fp32.txt 2>&1 || exit $?
find gpurun_out -name "*.csv" -size +5M -delete
