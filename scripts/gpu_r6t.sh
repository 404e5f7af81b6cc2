set -u
S=scripts/gpu_step.sh
bash $S r6t_dftw 200 python bench/dftw_rows.py || exit $?
