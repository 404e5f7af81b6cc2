"""FourCastNet AFNO fused spectral kernel (FFT_H -> block MLP on MFMA -> softshrink -> IFFT_H)
on [32, 90, 46, 768] bf16 spectra; prints us per call and achieved HBM GB/s.

Usage: python bench/bench_afno_spec.py [--batch 32]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from bench.bench_fft import time_graph  # noqa: E402
from tensorrt_dft_plugins_amd.ops import spectral as S  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args(argv)
    tdp.load_plugins()
    B, H, KM, C, nb = a.batch, 90, 46, 768, 8
    g = torch.Generator().manual_seed(0)
    bs = C // nb
    w1, w2 = 0.02 * torch.randn(2, nb, bs, bs, generator=g), 0.02 * torch.randn(2, nb, bs, bs, generator=g)
    b1, b2 = 0.02 * torch.randn(2, nb, bs, generator=g), 0.02 * torch.randn(2, nb, bs, generator=g)
    r = {}
    for split in (False, True):  # bf16 MFMA operands / bf16x3 split (fp32 spectrum)
        w1t, w2t, b1p, b2p = [t.cuda() for t in S.pack_afno_weights(w1, b1, w2, b2, split=split)]
        xw = torch.randn(B, H, KM, C, 2, device="cuda").to(torch.float32 if split else torch.bfloat16)
        f = lambda: torch.ops.amd_dft.afno_spectral(xw, w1t, w2t, b1p, b2p, 0.01)  # noqa: E731
        f()
        t = min(time_graph(f, 10) for _ in range(5))
        tag = "fp32_x3" if split else "bf16"
        r[tag] = {"us": round(t, 1), "GBps": round(2 * xw.numel() * xw.element_size() / t / 1e3, 1)}
    print(json.dumps(r))
    return r


if __name__ == "__main__":
    main()
