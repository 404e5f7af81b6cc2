set -u
S=scripts/gpu_step.sh
bash $S r6f_stamps 300 ./stampbin/gemm_stamps || exit $?
bash $S r6f_gemm 400 python bench/bench_gemm.py --rounds 3 || exit $?
