"""fp32 FourCastNet comparators on one MI355X: eager PyTorch (rocFFT + hipBLASLt fp32 GEMMs,
torch backend), the amd backend, and the fp32 / bf16 GEMM rates on the MLP shapes.

Usage: python bench/probe_fp32.py [--batch 32] [--depth 12] [--steps 3]
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from bench.bench_fft import time_graph  # noqa: E402
from tensorrt_dft_plugins_amd.engine.capture import CapturedModule  # noqa: E402
from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet  # noqa: E402


def step_ms(model, x, steps, graph=True):
    cap = CapturedModule(model, [x], use_graph=graph)
    cap.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        cap.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1000.0 / steps


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args(argv)
    tdp.load_plugins()
    out = {}
    M, C, Hd = 32 * 16200, 768, 3072
    x = torch.randn(M, C, device="cuda")
    w1 = torch.randn(Hd, C, device="cuda") * 0.02
    b1 = torch.randn(Hd, device="cuda") * 0.02
    flop = 2.0 * M * C * Hd
    for name, dt in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
        xx, ww, bb = x.to(dt), w1.to(dt), b1.to(dt)
        us = time_graph(lambda: F.linear(xx, ww, bb), 3)
        out[f"fc1_{name}_hipblaslt_us"] = round(us, 1)
        out[f"fc1_{name}_hipblaslt_tflops"] = round(flop / us / 1e6, 1)
        print(name, out, flush=True)
    del x, w1
    torch.cuda.empty_cache()
    cfg = AFNOConfig(depth=a.depth)
    torch.manual_seed(0)
    inp = torch.randn(a.batch, cfg.in_chans, *cfg.img_size, device="cuda")
    for backend in ("torch", "amd"):
        m = AFNONet(cfg, backend=backend).cuda().eval()
        ms = step_ms(m, inp, a.steps)
        out[f"fourcastnet_fp32_{backend}_ms"] = round(ms, 2)
        out[f"fourcastnet_fp32_{backend}_samples_per_s"] = round(a.batch * 1000.0 / ms, 2)
        print(out, flush=True)
        del m
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
