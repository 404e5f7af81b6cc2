"""RCCL all-gather / all-to-all sweep over xGMI (the batch-DP output gather, SURVEY §2.5 C-1 /
§5.8; ``--op all_to_all`` is the slab-FFT transpose of parallel/slab_fft.py).

One process per GPU:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
      --master-port 29511 bench/bench_rccl.py [--dtype bf16] [--mb 1 4 16 64 166 332]
Rank 0 prints one JSON line per size: per-rank shard MB, time, algorithm bandwidth (gathered
bytes / time) and bus bandwidth ((world-1)/world * gathered bytes / time, the ring's per-link
traffic).  1327 MB is bench.py's per-rank output shard (batch 32 x 20 x 720 x 1440 bf16).
Without GPUs it runs on gloo (plumbing check only).
"""
import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorrt_dft_plugins_amd.parallel import all_gather_batch, init_distributed, world_info  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, nargs="+", default=[1, 4, 16, 64, 166, 332, 1327])
    ap.add_argument("--op", default="all_gather", choices=["all_gather", "all_to_all", "ipc_gather"],
                    help="ipc_gather: direct pushes into every peer's buffer (parallel/ipc_gather.py)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args(argv)
    gpu = torch.cuda.is_available()
    # MI_DFT_DIST_BACKEND=gloo rehearses several ranks on one GPU (RCCL refuses that)
    init_distributed(os.environ.get("MI_DFT_DIST_BACKEND") or ("nccl" if gpu else "gloo"))
    rank, world = world_info()
    local = int(os.environ.get("LOCAL_RANK", 0))
    dev = torch.device("cuda", local % torch.cuda.device_count()) if gpu else torch.device("cpu")
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    es = torch.finfo(dt).bits // 8
    for mb in a.mb:
        n = max(1, int(mb * 1e6 / es))
        if a.op == "ipc_gather":  # direct-mesh pushes + host handshake + IPC events
            from tensorrt_dft_plugins_amd.parallel import IpcAllGather

            x = torch.randn(n, device=dev).to(dt)
            ig = IpcAllGather([n], dt, dev, nbuf=2)
            it = {"k": 0}

            def coll():
                ig.gather(x, it["k"])
                it["k"] += 1
        elif a.op == "all_to_all":  # n elements per peer block
            x = torch.randn(world * n, device=dev).to(dt)
            out = torch.empty(world * n, device=dev, dtype=dt)

            def coll():
                dist.all_to_all_single(out, x)
        else:
            x = torch.randn(n, device=dev).to(dt)
            out = torch.empty(world * n, device=dev, dtype=dt)

            def coll():
                all_gather_batch(x, out)
        for _ in range(3):
            coll()
        if gpu:
            torch.cuda.synchronize()
        dist.barrier()
        if gpu:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                coll()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
        else:
            import time

            t0 = time.perf_counter()
            for _ in range(a.iters):
                coll()
            ms = (time.perf_counter() - t0) * 1e3 / a.iters
        t = torch.tensor([ms], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
        total = world * n * es
        if rank == 0:
            print(json.dumps({"op": a.op, "world": world, "dtype": a.dtype, "shard_MB": round(n * es / 1e6, 3), "ms": round(ms, 4),
                              "algbw_GBps": round(total / (ms * 1e-3) / 1e9, 2),
                              "busbw_GBps": round((world - 1) / world * total / (ms * 1e-3) / 1e9, 2),
                              "backend": "ipc" if a.op == "ipc_gather" else dist.get_backend()}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
