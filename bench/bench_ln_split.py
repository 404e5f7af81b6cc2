"""LN2 -> split-pair kernel (layer_norm_split, fp32 FourCastNet path) on [32*16200, 768]: graph
time, bytes/s, and error vs an fp64 LayerNorm.  MI_DFT_LN_SPLIT=dup selects the older
duplicated-load kernel for A/B.   Usage: python bench/bench_ln_split.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from bench.bench_fft import time_graph  # noqa: E402
from tensorrt_dft_plugins_amd.ops.spectral import unsplit_bf16  # noqa: E402


def main():
    tdp.load_plugins()
    ops = torch.ops.amd_dft
    torch.manual_seed(0)
    M, C = 32 * 16200, 768
    x = torch.randn(M, C, device="cuda") * 2 + 0.5
    g = torch.rand(C, device="cuda") + 0.5
    b = torch.randn(C, device="cuda") * 0.1
    pre = torch.randn(C, device="cuda") * 0.1
    for name, p in (("no pre", None), ("pre", pre)):
        us = min(time_graph(lambda: ops.layer_norm_split(x, g, b, 1e-6, p), 10) for _ in range(5))
        y = ops.layer_norm_split(x[:4096], g, b, 1e-6, p)
        xx = x[:4096].double() + (0 if p is None else p.double())
        ref = torch.nn.functional.layer_norm(xx, (C,), g.double(), b.double(), 1e-6)
        err = ((unsplit_bf16(y).double() - ref).norm() / ref.norm()).item()
        print(f"layer_norm_split {name:6s} {os.environ.get('MI_DFT_LN_SPLIT', 'lds'):4s}: {us:8.1f} us  "
              f"{2 * M * C * 4 / us / 1e6:6.2f} TB/s  rel err {err:.2e}", flush=True)
    # cold: rotate over 4 distinct inputs / outputs (12.8 GB > the 256 MB Infinity Cache)
    xs = [torch.randn(M, C, device="cuda") for _ in range(4)]
    it = {"i": 0}

    def cold():
        i = it["i"] % 4
        ops.layer_norm_split(xs[i], g, b, 1e-6, None)
        it["i"] += 1

    us = min(time_graph(cold, 8) for _ in range(5))
    print(f"layer_norm_split cold (4 rotating inputs): {us:8.1f} us  {2 * M * C * 4 / us / 1e6:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import note_tuning_build

    note_tuning_build("MI_DFT_LN_SPLIT")
    main()
