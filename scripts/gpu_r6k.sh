set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
bash $S r6k_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
bash $S r6k_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
bash $S r6k_bench 600 python bench.py --json-out gpurun_out/r6k_bench.json || exit $?
for i in 1 2; do
  bash $S r6k_fno_new_$i 200 python bench/bench_fno.py --amd-only --rounds 10 || exit $?
  MI_DFT_LIB=ab/actsc_C.so bash $S r6k_fno_sc_$i 200 python bench/bench_fno.py --amd-only --rounds 10 || exit $?
  MI_DFT_LIB=ab/acttanh_C.so bash $S r6k_fno_tanh_$i 200 python bench/bench_fno.py --amd-only --rounds 10 || exit $?
done
PROF_TAG=_r6k_fp32 BENCH_ARGS="--native-steps 0" bash scripts/prof_bench.sh > gpurun_out/r6k_prof_fp32.txt 2>&1 || exit $?
find gpurun_out -name "*.csv" -size +5M -delete
