set -u
S=scripts/gpu_step.sh
bash $S r6g_fg_rccl 600 python bench.py --force-gather --extra-steps 0 --native-steps 0 --json-out gpurun_out/r6g_fg_rccl.json || exit $?
bash $S r6g_fg_ipc 600 python bench.py --force-gather --gather ipc --no-fft --extra-steps 0 --native-steps 0 --json-out gpurun_out/r6g_fg_ipc.json || exit $?
