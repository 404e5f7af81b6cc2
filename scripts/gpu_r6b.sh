set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
bash $S r6b_diff 400 python bench/engine_diff.py --rounds 6 || exit $?
bash $S r6b_prof_contrib 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6b_prof_contrib -o run -- python bench/engine_diff.py --export contrib --rounds 1 --iters 5 || exit $?
bash $S r6b_prof_amd 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6b_prof_amd -o run -- python bench/engine_diff.py --export amd --rounds 1 --iters 5 || exit $?
