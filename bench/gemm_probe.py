"""Runs the hand GEMM (and hipBLASLt) on the FourCastNet MLP shapes a few times, for rocprofv3
counter passes (scripts/pmc_cmd.sh).  Usage: python bench/gemm_probe.py [--iters 3] [--blas]"""
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
for _ in range(a.iters):
    ops.linear(x, w1, b1, 1, None)
    ops.linear(x, w1, b1, 0, None)
    ops.linear(h, w2, b2, 0, None)
    if a.blas:
        F.linear(x, w1, b1.bfloat16())
        F.linear(h, w2, b2.bfloat16())
torch.cuda.synchronize()
print("ok")
