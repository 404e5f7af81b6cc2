"""FNO SpectralConv2d block (BASELINE config 3: rfft2 -> complex mode mix -> irfft2, + 1x1 conv
+ GELU), 20 ch, 720x1440, bf16 (and fp32): native kernels vs the eager PyTorch block (torch.fft
= rocFFT + einsum + conv2d, comparator only), both eager and hipGraph-captured, interleaved
rounds in one process.

Usage: python bench/bench_fno.py [--batch 1] [--modes 32 32] [--width 20] [--rounds 10] [--json out.json]
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from bench.bench_fft import time_eager, time_graph  # noqa: E402
from tensorrt_dft_plugins_amd.models.fno import FNOBlock, fno_block_flops  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", type=int, nargs=2, default=[720, 1440])
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--width", type=int, default=20)
    ap.add_argument("--modes", type=int, nargs=2, default=[32, 32])
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json", default=None)
    ap.add_argument("--amd-only", action="store_true", help="skip the torch comparator (profiling)")
    a = ap.parse_args(argv)
    tdp.load_plugins()
    dev = torch.device("cuda:0")
    H, W = a.shape
    torch.manual_seed(0)
    blk = FNOBlock(a.width, a.modes[0], a.modes[1], backend="torch").to(dev).eval()
    amd = FNOBlock(a.width, a.modes[0], a.modes[1], backend="amd").to(dev).eval()
    amd.load_state_dict(blk.state_dict())
    res = {"shape": [a.batch, a.width, H, W], "modes": a.modes}
    for dt in (torch.bfloat16, torch.float32):
        x = torch.randn(a.batch, a.width, H, W, device=dev).to(dt)
        blk_t = copy.deepcopy(blk).to(dt)  # eager comparator in the same dtype
        with torch.no_grad():
            ref = blk(x.float())
            out = amd(x)
        err = float((out.float() - ref).norm() / ref.norm())
        tag = "bf16" if dt == torch.bfloat16 else "fp32"
        samples = {"amd_eager": [], "amd_graph": [], "torch_eager": [], "torch_graph": []}
        with torch.no_grad():
            for _ in range(a.rounds):
                samples["amd_eager"].append(time_eager(lambda: amd(x), a.iters))
                samples["amd_graph"].append(time_graph(lambda: amd(x), a.iters))
                if not a.amd_only:
                    samples["torch_eager"].append(time_eager(lambda: blk_t(x), a.iters))
                    samples["torch_graph"].append(time_graph(lambda: blk_t(x), a.iters))
        r = {k: {"median_us": statistics.median(v), "min_us": min(v)} for k, v in samples.items() if v}
        r["rel_l2_vs_fp32_torch"] = err
        if not a.amd_only:
            r["speedup_graph_vs_torch"] = r["torch_graph"]["median_us"] / r["amd_graph"]["median_us"]
        fl = fno_block_flops(a.batch, a.width, H, W, *a.modes)
        r["block_gflops_amd_graph"] = fl / (r["amd_graph"]["median_us"] * 1e3)
        nbytes = x.element_size() * x.numel()
        # minimum HBM traffic: read x twice (FFT + pointwise), write y once (+ spectral output round trip)
        r["hbm_GBps_amd_graph"] = 5 * nbytes / (r["amd_graph"]["median_us"] * 1e3)
        res[tag] = r
        print(tag, json.dumps(r), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)
    return res


if __name__ == "__main__":
    main()
