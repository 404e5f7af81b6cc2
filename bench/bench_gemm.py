"""Hand-written fused-epilogue GEMM vs hipBLASLt (torch) on the FourCastNet MLP shapes,
interleaved rounds in one process.

Usage: python bench/bench_gemm.py [--rows 518400] [--x3]
(MI_DFT_GEMM_PERSIST=1: the fp32 block's GEMMs on the persistent grid -- run once with each to A/B)
"""
import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from bench.bench_fft import time_graph  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32 * 16200)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--x3", action="store_true", help="bf16x3 split GEMMs (fp32 path) + the bf16 hand GEMMs")
    ap.add_argument("--iters", type=int, default=3, help="calls per captured graph (sustained-load check: e.g. 30)")
    ap.add_argument("--zero-lo", action="store_true",
                    help="x3: split bf16-representable operands (lo planes all zero) -- the pre-round-3 harness; "
                         "zero lo halves draw less MFMA power, so the clock and the time are optimistic")
    a = ap.parse_args(argv)
    tdp.load_plugins()
    M, C, Hd = a.rows, 768, 3072
    dev = "cuda"
    x = torch.randn(M, C, device=dev).to(torch.bfloat16)
    h = torch.randn(M, Hd, device=dev).to(torch.bfloat16)
    w1 = (torch.randn(Hd, C, device=dev) * 0.02).to(torch.bfloat16)
    w2 = (torch.randn(C, Hd, device=dev) * 0.02).to(torch.bfloat16)
    b1 = (torch.randn(Hd, device=dev) * 0.02)
    b2 = (torch.randn(C, device=dev) * 0.02)
    b1h, b2h = b1.to(torch.bfloat16), b2.to(torch.bfloat16)
    ops = torch.ops.amd_dft
    st_b = ops.ln_stats(x.float(), None, 1e-6)
    c1_b = torch.randn(Hd, device=dev)
    rb = torch.randn(M, C, device=dev).to(torch.bfloat16)
    v = {
        "fc1_gelu amd": lambda: ops.linear(x, w1, b1, 1, None),
        # hipBLASLt's GELU epilogue is the tanh form: the like-for-like hand kernel is act 2
        "fc1_gelu_tanh amd": lambda: ops.linear(x, w1, b1, 2, None),
        "fc1_gelu hipblaslt": lambda: torch._addmm_activation(b1h, x, w1.t(), use_gelu=True),
        "fc1 amd": lambda: ops.linear(x, w1, b1, 0, None),
        "fc1 hipblaslt": lambda: F.linear(x, w1, b1h),
        "fc2 amd": lambda: ops.linear(h, w2, b2, 0, None),
        "fc2 hipblaslt": lambda: F.linear(h, w2, b2h),
        # the bf16 block's forms (persistent variants under MI_DFT_GEMM_PERSIST=1)
        "fc1_gelu amd LN": lambda: ops.linear_ln(x, w1, c1_b, b1, st_b, 1),
        "fc1_gelu_tanh amd LN": lambda: ops.linear_ln(x, w1, c1_b, b1, st_b, 2),
        "fc2 amd (+res)": lambda: ops.linear(h, w2, b2, 0, rb),
        # the model's fc2: bias pending into the next block, + the next LN's partial statistics
        "fc2 amd (+res, no bias)": lambda: ops.linear(h, w2, None, 0, rb),
        "fc2 amd (+res, stats)": lambda: ops.linear_stats(h, w2, rb, b2),
    }
    if a.x3:
        # full fp32 operands (non-zero lo halves, as the model's activations and weights have)
        src = (x.float(), h.float(), w1.float(), w2.float())
        if not a.zero_lo:
            src = (torch.randn(M, C, device=dev), F.gelu(torch.randn(M, Hd, device=dev)),
                   torch.randn(Hd, C, device=dev) * 0.02, torch.randn(C, Hd, device=dev) * 0.02)
        xs, hs, w1s, w2s = (ops.split_bf16(t) for t in src)
        r32 = torch.randn(M, C, device=dev)
        st = ops.ln_stats(src[0], None, 1e-6)
        c1 = torch.randn(Hd, device=dev)
        v = {
            "fc1_gelu x3 (split out)": lambda: ops.linear3(xs, w1s, b1, 1, None, True),
            "fc2 x3 (+fp32 residual)": lambda: ops.linear3(hs, w2s, None, 0, r32, False),
            # the fp32 block's forms: LayerNorm folded into fc1; fc2 + the next LN's partial statistics
            "fc1_gelu x3 LN (split out)": lambda: ops.linear3_ln(xs, w1s, c1, b1, st, 1),
            "fc2 x3 (+residual, stats)": lambda: ops.linear3_stats(hs, w2s, r32, b2),
            "fc1_gelu amd": v["fc1_gelu amd"],
            "fc2 amd": v["fc2 amd"],
            "fc1_gelu amd LN": v["fc1_gelu amd LN"],
            "fc2 amd (+res)": v["fc2 amd (+res)"],
        }
    res = {k: [] for k in v}
    for _ in range(a.rounds):
        for k, f in v.items():
            res[k].append(time_graph(f, a.iters))
    flop = 2.0 * M * C * Hd
    out = {}
    for k, t in res.items():
        med = statistics.median(t)
        out[k] = {"us": round(med, 1), "TFLOPs": round(flop / med / 1e6, 1)}
        mult = 3 if "x3" in k else 1
        print(f"{k:26s} {med:9.1f} us  {flop / med / 1e6:7.1f} TFLOP/s  ({mult * flop / med / 1e6:7.1f} bf16-MFMA TFLOP/s)", flush=True)
    y = ops.linear(x[:4096], w1, b1, 1, None).float()
    ref = F.gelu(F.linear(x[:4096].float(), w1.float(), b1))
    print("rel err", ((y - ref).norm() / ref.norm()).item())
    yt = ops.linear(x[:4096], w1, b1, 2, None).float()
    print("rel err tanh form vs erf reference", ((yt - ref).norm() / ref.norm()).item(),
          "vs tanh reference", ((yt - F.gelu(F.linear(x[:4096].float(), w1.float(), b1), approximate="tanh")).norm()
                                / ref.norm()).item())
    return out


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import note_tuning_build

    note_tuning_build("MI_DFT_GEMM_PERSIST")
    main()
