"""fp32 FourCastNet AFNO C2R epilogue (c2r_ln_add_split: C2R_W + skips + LN2 partials + bf16x3 split pairs of the
residual stream) on [32, 90, 180, 768] per out_mode (1: + the fp32 residual-stream output, 0: pairs only,
2: + the bf16 third split term instead of the fp32 output); us per call.

Usage: python bench/bench_c2r_split.py [--batch 32]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from bench.bench_fft import time_graph  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args(argv)
    tdp.load_plugins()
    B, H, W, KM, C = a.batch, 90, 180, 46, 768
    dev = "cuda"
    X = torch.randn(B, H, KM, C, 2, device=dev)
    x = torch.randn(B, H, W, C, device=dev)
    st = torch.stack([0.1 * torch.randn(B * H * W, device=dev), torch.rand(B * H * W, device=dev) + 0.5], 1)
    g, b = torch.rand(C, device=dev) + 0.5, 0.1 * torch.randn(C, device=dev)
    ops = torch.ops.amd_dft
    r = {}
    for mode in (1, 0, 2, 1, 0, 2):
        f = lambda: ops.c2r_ln_add_split(X, 2, W, 1.0 / 16200 ** 0.5, x, st, g, b, None, mode)  # noqa: E731
        f()
        r.setdefault(f"out_mode={mode}", []).append(round(min(time_graph(f, 10) for _ in range(3)), 1))
    print(json.dumps(r))


if __name__ == "__main__":
    main()
