"""Probe: FourCastNet (720x1440, depth 12) batch 32 run as sequential micro-batches inside one
hipGraph, so that a block's producer -> consumer activations (c * 50 MB fp32 per sample) can
stay in the 256 MB Infinity Cache instead of round-tripping HBM.  Same FLOPs, same outputs.

Usage: python bench/microbatch_probe.py [--dtype fp32|bf16] [--chunks 32,8,4,2,1]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--chunks", default="32,8,4,2,1")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args(argv)
    tdp.load_plugins()
    dt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    torch.manual_seed(0)
    cfg = AFNOConfig()
    m = AFNONet(cfg, backend="amd").cuda().to(dt).eval()
    B = a.batch
    x = torch.randn(B, cfg.in_chans, *cfg.img_size, device="cuda").to(dt)
    out = torch.empty(B, cfg.out_chans, *cfg.img_size, device="cuda", dtype=dt)
    ref = None
    for c in [int(v) for v in a.chunks.split(",")]:
        def fn():
            for i in range(0, B, c):
                out[i:i + c].copy_(m(x[i:i + c]))

        with torch.no_grad():
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                fn()
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                fn()
            g.replay()
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            if ref is None:
                ref = out.clone()
                d = 0.0
            else:
                d = ((out.float() - ref.float()).norm() / ref.float().norm()).item()
        ms = sorted(ts)[len(ts) // 2]
        print(f"{a.dtype} chunk {c:2d}: {ms:8.2f} ms/step  {B / ms * 1e3:7.1f} samples/s  rel diff vs chunk {a.chunks.split(',')[0]}: {d:.2e}",
              flush=True)
        del g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
