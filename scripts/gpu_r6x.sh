set -u
S=scripts/gpu_step.sh
bash $S r6x_mem 400 python bench/export_mem.py || exit $?
bash scripts/gpu_r6w.sh || exit $?
