"""Why is the fp32 AFNO H-filter (afno_spectral_x3) slower inside the FourCastNet step than
standalone?  (851 us in the step vs 741-751 us standalone.)

One workload, three contexts for the same kernel at the same shape [32, 90, 46, 768]:
  step      the fp32 model (depth --depth, batch 32) replayed as one hipGraph: the filter runs
            between afno_w_r2c_ln and afno_w_c2r_ln, right after the previous block's MLP GEMMs
  captured  the filter alone, replayed --calls times in a hipGraph, on the spectrum the model's
            block 0 actually produced (same data, no GEMM neighbours)
  random    the filter alone on N(0, s^2) spectra, s = the captured spectrum's rms (same
            magnitude, different values: the standalone bench's setting); ``random1``: s = 1
  gemmgap   the captured-data filter with one model fc1 GEMM (bf16x3, M = 518400) before every
            call inside the same graph: the step's neighbourhood without the rest of the model
Run it under ``rocprofv3 --kernel-trace --stats`` (durations) and under ``--pmc`` passes (cycles per
wave, GRBM_GUI_ACTIVE per dispatch -> clock) to separate clock, data and co-residency effects.

  python bench/afno_gap.py --mode step|captured|random|random1|gemmgap [--depth 4] [--calls 8]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet  # noqa: E402
from tensorrt_dft_plugins_amd.ops import spectral as S  # noqa: E402


def graph_of(fn, n):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    return g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", required=True, choices=["step", "captured", "random", "random1", "gemmgap"])
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--calls", type=int, default=8)
    ap.add_argument("--replays", type=int, default=3)
    a = ap.parse_args()
    tdp.load_plugins()
    torch.manual_seed(0)
    cfg = AFNOConfig(depth=a.depth)
    m = AFNONet(cfg, backend="amd").cuda().eval()
    x = torch.randn(32, cfg.in_chans, *cfg.img_size, device="cuda")
    seen = {}
    orig = S.afno_spectral_h

    def spy(xw, w1, b1, w2, b2, nb, lam, owner=None):
        if "xw" not in seen:
            seen["xw"] = xw.clone()
            seen["args"] = (w1, b1, w2, b2, nb, lam, owner)
        return orig(xw, w1, b1, w2, b2, nb, lam, owner=owner)

    S.afno_spectral_h = spy
    with torch.no_grad():
        m(x)
    S.afno_spectral_h = orig
    torch.cuda.synchronize()
    xw = seen["xw"]
    w1, b1, w2, b2, nb, lam, owner = seen["args"]
    rms = float(xw.float().pow(2).mean().sqrt())
    print(f"[gap] captured spectrum {list(xw.shape)} {xw.dtype} rms {rms:.4g}", file=sys.stderr, flush=True)
    with torch.no_grad():
        if a.mode == "step":
            g = graph_of(lambda: m(x), 1)
        else:
            if a.mode == "captured" or a.mode == "gemmgap":
                inp = xw
            else:
                inp = torch.randn_like(xw) * (rms if a.mode == "random" else 1.0)
            f = lambda: orig(inp, w1, b1, w2, b2, nb, lam, owner=owner)  # noqa: E731
            if a.mode == "gemmgap":
                blk = m.blocks[1]
                hid_in = torch.randn(32 * cfg.h * cfg.w, 2 * cfg.embed_dim, device="cuda").to(torch.bfloat16)
                ws = S.split_bf16(blk.mlp.fc1.weight)
                ops = torch.ops.amd_dft

                def f2():
                    ops.linear3(hid_in, ws, blk.mlp.fc1.bias.float(), 1, None, True)
                    f()
                g = graph_of(f2, a.calls)
            else:
                g = graph_of(f, a.calls)
        torch.cuda.synchronize()
        for _ in range(a.replays):
            t0 = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            print(f"[gap] {a.mode}: replay {1e3 * (time.perf_counter() - t0):.2f} ms", file=sys.stderr, flush=True)
    print("afno_gap done")


if __name__ == "__main__":
    main()
