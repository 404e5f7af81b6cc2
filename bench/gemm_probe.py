"""Runs the hand GEMM (and hipBLASLt) on the FourCastNet MLP shapes a few times, for rocprofv3
counter passes (scripts/pmc_cmd.sh).  Usage: python bench/gemm_probe.py [--iters 3] [--blas] [--x3]"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--rows", type=int, default=32 * 16200)
ap.add_argument("--blas", action="store_true")
ap.add_argument("--x3", action="store_true", help="only the bf16x3 (fp32-path) fc1 + GELU -> fc2 + residual pair")
a = ap.parse_args()
tdp.load_plugins()
M, C, Hd = a.rows, 768, 3072
x = torch.randn(M, C, device="cuda").to(torch.bfloat16)
h = torch.randn(M, Hd, device="cuda").to(torch.bfloat16)
w1 = (torch.randn(Hd, C, device="cuda") * 0.02).to(torch.bfloat16)
w2 = (torch.randn(C, Hd, device="cuda") * 0.02).to(torch.bfloat16)
b1 = torch.randn(Hd, device="cuda") * 0.02
b2 = torch.randn(C, device="cuda") * 0.02
ops = torch.ops.amd_dft
if a.x3:
    xs = ops.split_bf16(x.float())
    w1s, w2s = ops.split_bf16(w1.float()), ops.split_bf16(w2.float())
    r32 = torch.randn(M, C, device="cuda")
    for _ in range(a.iters):
        hs = ops.linear3(xs, w1s, b1, 1, None, True)
        ops.linear3(hs, w2s, None, 0, r32, False)
    torch.cuda.synchronize()
    print("ok")
    sys.exit(0)
for _ in range(a.iters):
    ops.linear(x, w1, b1, 1, None)
    ops.linear(x, w1, b1, 0, None)
    ops.linear(h, w2, b2, 0, None)
    if a.blas:
        F.linear(x, w1, b1.bfloat16())
        F.linear(h, w2, b2.bfloat16())
torch.cuda.synchronize()
print("ok")
