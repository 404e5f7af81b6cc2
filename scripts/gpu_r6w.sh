set -u
S=scripts/gpu_step.sh
# two ranks sharing the one GPU over Gloo: the bench's world > 1 path end to end (full model, batch 8 per rank:
# the contrib export trace holds ~170 GB at batch 32, one GPU cannot hold two) (engine builds on every
# rank, native-export extra timed before the headline with both runners alive, gather + its verification)
MI_DFT_DIST_BACKEND=gloo bash $S r6w_gloo2 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --batch 8 --steps 2 --warmup 1 --native-steps 2 --extra-steps 0 \
  --no-fft --json-out gpurun_out/r6w_gloo2.json || exit $?
