set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
bash $S r6e_tests 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
bash $S r6e_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
bash $S r6e_bench 600 python bench.py --json-out gpurun_out/r6e_bench.json || exit $?
PROF_TAG=_r6e_bf16 BENCH_ARGS="--dtype bf16" bash scripts/prof_bench.sh > gpurun_out/r6e_prof_bf16.txt 2>&1 || exit $?
find gpurun_out -name "*.csv" -size +5M -delete
