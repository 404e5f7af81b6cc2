"""Workload for rocprofv3 PMC passes (scripts/pmc_targets.sh): one call of every headline kernel.

rfft2 / irfft2 720x1440 fp32 (row + column kernels), the FNO block (BASELINE config 3, bf16), and a
depth-2 FourCastNet forward at batch 32 in fp32 (bf16x3 GEMMs, fp32 H-filter) and bf16 -- depth 2
covers every per-block kernel (first block: ln_stats; last block: the split-pair head operand).
A warm-up call of each runs first so the counted calls see built plans and packed weights.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet  # noqa: E402
from tensorrt_dft_plugins_amd.models.fno import FNOBlock  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=2)
    ap.add_argument("--depth", type=int, default=2)
    ap.add_argument("--only", default="fft,fno,fp32,bf16")
    a = ap.parse_args()
    tdp.load_plugins()
    only = set(a.only.split(","))
    torch.manual_seed(0)
    with torch.no_grad():
        if "fft" in only:
            x = torch.randn(1, 720, 1440, device="cuda")
            y = tdp.contrib_rfft(x, signal_ndim=2)
            for _ in range(a.calls):
                tdp.contrib_rfft(x, signal_ndim=2)
                tdp.contrib_irfft(y, signal_ndim=2)
        if "fno" in only:
            blk = FNOBlock(20, 32, 32, backend="amd").cuda().eval()
            xb = torch.randn(1, 20, 720, 1440, device="cuda").to(torch.bfloat16)
            for _ in range(a.calls + 1):
                blk(xb)
        for tag, dt in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
            if tag not in only:
                continue
            cfg = AFNOConfig(depth=a.depth)
            m = AFNONet(cfg, backend="amd").cuda().to(dt).eval()
            xi = torch.randn(32, cfg.in_chans, *cfg.img_size, device="cuda").to(dt)
            for _ in range(2):
                m(xi)
            del m, xi
            torch.cuda.empty_cache()
        torch.cuda.synchronize()
    print("pmc_targets done")


if __name__ == "__main__":
    main()
