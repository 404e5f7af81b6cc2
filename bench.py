"""Headline benchmark (driver contract): FourCastNet AFNO batch-DP inference samples/s on N
MI355X GPUs (one process per GPU, RCCL all-gather of the outputs over xGMI, hipGraph-captured
per-step forward), plus the rfft2 / irfft2 720x1440 fp32 single-op latency (us).

Metric/config from BASELINE.json: "rfft2 720x1440 us + FourCastNet-FNO samples/sec at 1/2/4/8
MI355X"; FourCastNet AFNO (720x1440, patch 8, embed 768, depth 12, 8 AFNO blocks), batch 32
per GPU (weak scaling), bf16 activations/weights (FFTs fp32 internally), synthetic inputs,
random-init weights.  Every timed step runs the full forward (all 12 blocks) and the output
all-gather; K steps are bracketed by barrier + synchronize, the max over ranks is reported.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet, flops_per_sample  # noqa: E402
from tensorrt_dft_plugins_amd.parallel import DataParallelInference, init_distributed, world_info  # noqa: E402

METRIC = "rfft2 720×1440 µs + FourCastNet-FNO samples/sec at 1/2/4/8 MI355X"


def log(msg: str) -> None:
    rank = int(os.environ.get("RANK", "0"))
    if rank == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def time_fft_us(iters: int = 50, rounds: int = 5) -> dict:
    """rfft2 / irfft2 720x1440 fp32 batch 1 (contrib Rfft/Irfft ops), hipGraph of `iters` calls."""
    x = torch.randn(1, 720, 1440, device="cuda")
    y = tdp.contrib_rfft(x, signal_ndim=2)
    res = {}
    for name, fn in (("rfft2_720x1440_us", lambda: tdp.contrib_rfft(x, signal_ndim=2)),
                     ("irfft2_720x1440_us", lambda: tdp.contrib_irfft(y, signal_ndim=2))):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g):
            for _ in range(iters):
                fn()
        ts = []
        for _ in range(rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1000.0 / iters)
        res[name] = round(sorted(ts)[len(ts) // 2], 3)
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="samples per GPU (weak scaling)")
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--no-fft", action="store_true", help="skip the rfft2 720x1440 latency probe")
    ap.add_argument("--tiny", action="store_true", help="tiny model/grid (harness smoke test, CPU ok)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--streams", type=int, default=1, help="micro-batches on concurrent HIP streams per GPU")
    ap.add_argument("--no-gemm-table", action="store_true",
                    help="hipBLASLt default heuristics instead of tensorrt_dft_plugins_amd/tuning/*.csv")
    a = ap.parse_args(argv)

    rank, world, local = init_distributed()
    if world != a.gpus and world > 1:
        log(f"note: --gpus {a.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    cuda = torch.cuda.is_available()
    # local % count: lets a Gloo rehearsal (MI_DFT_DIST_BACKEND=gloo) put several ranks on one GPU
    dev = torch.device("cuda", local % torch.cuda.device_count()) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(dev)
    tdp.load_plugins()
    torch.manual_seed(1234 + rank)
    gemm_table = None
    if cuda and not a.no_gemm_table:
        # one GPU: fastest hipBLASLt solutions; DP: no stream-K GEMMs, which stall while the
        # all-gather's RCCL blocks hold CUs (tensorrt_dft_plugins_amd/utils/gemm_tables.py)
        from tensorrt_dft_plugins_amd.utils.gemm_tables import table_for_world, use_gemm_table

        path = table_for_world(world)
        if use_gemm_table(path):
            gemm_table = os.path.basename(path)
        log(f"GEMM solution table: {gemm_table}")

    if a.tiny:
        cfg = AFNOConfig(img_size=(48, 96), in_chans=4, out_chans=4, embed_dim=64, depth=2, num_blocks=4)
    else:
        cfg = AFNOConfig(depth=a.depth)
    dtype = torch.bfloat16 if cuda else torch.float32
    model = AFNONet(cfg, backend="amd").to(dev).to(dtype).eval()
    B = a.batch if not a.tiny else min(a.batch, 2)
    x = torch.randn(B, cfg.in_chans, *cfg.img_size, device=dev).to(dtype)

    fft = {}
    if cuda and not a.no_fft and not a.tiny and rank == 0:
        fft = time_fft_us()
        log(f"fft probe: {fft}")

    t_build = time.perf_counter()
    model.micro_batches = max(1, a.streams)
    runner = DataParallelInference(model, x, gather=not a.no_gather, use_graph=not a.no_graph)
    log(f"captured forward (graph={runner.cap.use_graph}) in {time.perf_counter() - t_build:.1f}s; "
        f"world={world} batch/GPU={B}")

    def sync():
        if cuda:
            torch.cuda.synchronize(dev)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(a.warmup):
        runner.step()
    runner.drain()
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        runner.step()
    runner.drain()
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if cuda else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = elapsed * 1000.0 / a.steps
    samples_per_s = world * B / (elapsed / a.steps)
    tflops = samples_per_s * flops_per_sample(cfg) / 1e12
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(samples_per_s, 3),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
            "data": "synthetic inputs, random-init weights",
            "config": {
                "model": "FourCastNet AFNO (720x1440, patch 8, embed 768, depth %d, 8 AFNO blocks)" % cfg.depth
                if not a.tiny else "tiny AFNO (harness test)",
                "global_batch": world * B,
                "seq_len": cfg.h * cfg.w,
                "parallelism": f"dp{world}",
                "per_gpu_batch": B,
                "hipgraph": runner.cap.use_graph,
                "output_allgather": runner.gather,
                "streams": a.streams,
                "gemm_table": gemm_table,
            },
            "model_tflops_per_s": round(tflops, 2),
        }
        out.update(fft)
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
