set -u
S=scripts/gpu_step.sh
bash $S r6p_stamps 120 ./ab/fno_stamps || exit $?
