"""rfft2 / irfft2 720x1440 fp32 batch-1 latency (us): hand-written Stockham kernels vs
torch.fft (rocFFT, comparator only), interleaved rounds in one process, eager and hipGraph.

Usage: python bench/bench_fft.py [--shape 720 1440] [--batch 1] [--rounds 20] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402


def time_graph(fn, iters: int) -> float:
    """us per call of fn, captured `iters` times into one hipGraph."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / iters


def time_eager(fn, iters: int) -> float:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / iters


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", type=int, nargs=2, default=[720, 1440])
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    H, W = a.shape
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    x = torch.randn(a.batch, H, W, device=dev)
    yc = torch.fft.rfft2(x)
    yr = torch.view_as_real(yc).contiguous()
    variants = {
        "amd_rfft2": lambda: tdp.contrib_rfft(x, signal_ndim=2),
        "amd_irfft2": lambda: tdp.contrib_irfft(yr, signal_ndim=2),
        "torch_rfft2": lambda: torch.fft.rfft2(x),
        "torch_irfft2": lambda: torch.fft.irfft2(yc),
    }
    res = {k: {"graph": [], "eager": []} for k in variants}
    for _ in range(a.rounds):
        for k, fn in variants.items():
            res[k]["graph"].append(time_graph(fn, a.iters))
            res[k]["eager"].append(time_eager(fn, a.iters))
    out = {"shape": [a.batch, H, W], "dtype": "fp32"}
    for k, v in res.items():
        out[k] = {m: {"median_us": statistics.median(t), "min_us": min(t)} for m, t in v.items()}
    print(json.dumps(out, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
