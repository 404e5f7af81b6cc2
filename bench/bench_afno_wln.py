"""FourCastNet AFNO LayerNorm-fused W-transforms (csrc/spectral/afno_wfft.hip) on
[32, 90, 180, 768] bf16: ln_stats, r2c_ln (LN1 on load + R2C_W, 46 modes), c2r_ln_add
(C2R_W + x' + LN1(x')); us per call and achieved HBM TB/s.

Usage: python bench/bench_afno_wln.py [--batch 32]
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
    ops = torch.ops.amd_dft
    B, H, W, C, KM = a.batch, 90, 180, 768, 46
    x = torch.randn(B, H, W, C, device="cuda").to(torch.bfloat16)
    pre = 0.1 * torch.randn(C, device="cuda")
    g = 1 + 0.1 * torch.randn(C, device="cuda")
    b = 0.1 * torch.randn(C, device="cuda")
    s = 1.0 / (H * W) ** 0.5
    st = ops.ln_stats(x, pre, 1e-6)
    X = ops.r2c_ln(x, 2, s, KM, st, g, b, pre, torch.bfloat16)
    fs = {
        "ln_stats": (lambda: ops.ln_stats(x, pre, 1e-6), x.numel() * 2 + st.numel() * 4),
        "r2c_ln": (lambda: ops.r2c_ln(x, 2, s, KM, st, g, b, pre, torch.bfloat16), x.numel() * 2 + X.numel() * 2),
        "c2r_ln_add": (lambda: ops.c2r_ln_add(X, 2, W, s, x, st, g, b, pre), X.numel() * 2 + 2 * x.numel() * 2),
    }
    res = {}
    for name, (f, nbytes) in fs.items():
        f()
        t = min(time_graph(f, 10) for _ in range(5))
        res[name] = {"us": round(t, 1), "TBps": round(nbytes / t / 1e6, 2)}
    print(json.dumps(res), flush=True)
    return res


if __name__ == "__main__":
    main()
