"""Micro-batch pipelining of the fp32 FourCastNet step across two HIP streams (experiment).

The fp32 step is ~80 % bf16x3 GEMMs (MFMA-bound, power-limited) and ~17 % memory / latency-bound
AFNO spectral kernels (afno_w_r2c_ln, afno_spectral_x3, afno_w_c2r_ln).  Splitting the batch into two
halves on two streams, the second started once the first has finished its patch embedding, lets one
half's spectral kernels run while the other half's GEMMs occupy the MFMAs.

  python bench/bench_mbatch.py --mode one|seq2|mb2 [--depth 12] [--batch 32] [--replays 5]

  one   the whole batch, one stream (what bench.py captures)
  seq2  two half batches one after the other on one stream (the batch-size effect alone)
  mb2   two half batches on two streams, the second offset by the first's patch embedding
All three are captured into one hipGraph each and replayed; prints ms per step and samples/s, and
the max abs difference of the output against ``one``.
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


def fwd_f32(m, x, after_embed=None):
    """AFNONet.forward's fp32 'amd' branch with a hook after the patch embedding."""
    cfg = m.cfg
    B, p = x.shape[0], cfg.patch_size
    pos = m.pos_embed.reshape(cfg.h * cfg.w, cfg.embed_dim)
    pe = m.patch_embed
    ws = S.module_cached(m, "embed_split", (pe.weight,), lambda: S.split_bf16(pe.weight.reshape(cfg.embed_dim, -1)))
    t = torch.ops.amd_dft.patch_linear3(x.contiguous(), ws, pe.bias, pos, p).reshape(B, cfg.h, cfg.w, cfg.embed_dim)
    if after_embed is not None:
        after_embed()
    pending = None
    n = len(m.blocks)
    for i, blk in enumerate(m.blocks):
        t, pending = S.afno_block_amd(blk, t, pending, split_out=i == n - 1)
    hb = None
    pending = S.pending_bias(pending)
    if pending is not None and pending.dim() == 1:
        hb = m._head_bias_cpp(pending)
    elif pending is not None:
        t = t + pending
    hw = m._head_weight_cpp()
    wsh = S.module_cached(m, "head_split", (hw,), lambda: S.split_bf16(hw))
    ts = t.pairs if isinstance(t, S.SplitRows) else S.split_bf16(t.reshape(-1, cfg.embed_dim))
    return torch.ops.amd_dft.linear_unpatch3(ts, wsh, hb, cfg.out_chans, cfg.h, cfg.w, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", required=True, choices=["one", "seq2", "mb2"])
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--replays", type=int, default=5)
    a = ap.parse_args()
    tdp.load_plugins()
    torch.manual_seed(0)
    cfg = AFNOConfig(depth=a.depth)
    m = AFNONet(cfg, backend="amd").cuda().eval()
    x = torch.randn(a.batch, cfg.in_chans, *cfg.img_size, device="cuda")
    h = a.batch // 2
    out = torch.empty(a.batch, cfg.out_chans, *cfg.img_size, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def step():
        if a.mode == "one":
            out.copy_(fwd_f32(m, x))
        elif a.mode == "seq2":
            out[:h].copy_(fwd_f32(m, x[:h]))
            out[h:].copy_(fwd_f32(m, x[h:]))
        else:
            cur = torch.cuda.current_stream()
            s1.wait_stream(cur)
            s2.wait_stream(cur)
            ev = torch.cuda.Event()
            with torch.cuda.stream(s1):
                ya = fwd_f32(m, x[:h], after_embed=lambda: ev.record(s1))
                out[:h].copy_(ya)
            with torch.cuda.stream(s2):
                s2.wait_event(ev)
                yb = fwd_f32(m, x[h:])
                out[h:].copy_(yb)
            cur.wait_stream(s1)
            cur.wait_stream(s2)

    with torch.no_grad():
        step()
        torch.cuda.synchronize()
        ref = fwd_f32(m, x).clone() if a.mode != "one" else out.clone()
        g = torch.cuda.CUDAGraph()
        sc = torch.cuda.Stream()
        sc.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(sc):
            step()
        torch.cuda.current_stream().wait_stream(sc)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            step()
        for _ in range(2):
            g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.replays):
            t0 = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ms = sorted(ts)[len(ts) // 2] * 1e3
        err = (out - ref).abs().max().item()
    print(f"{a.mode}: depth {a.depth} batch {a.batch}: median {ms:.2f} ms/step = {a.batch / ms * 1e3:.2f} samples/s "
          f"(min {min(ts) * 1e3:.2f}); max |out - one| = {err:.3e}", flush=True)


if __name__ == "__main__":
    main()
