"""Contrib-export engine vs native-export engine (FourCastNet fp32, 720x1440, depth 12, batch 32):
node sequences of both built graphs and interleaved hipGraph timings (ABAB), so a gap between the
two engines can be attributed to the nodes that differ.

  python bench/engine_diff.py [--depth 12] [--batch 32] [--rounds 4] [--iters 5] [--export both|contrib|amd]
With ``--export contrib`` / ``amd`` only that engine is built and replayed (``--iters`` x ``--rounds``),
e.g. under ``rocprofv3 --kernel-trace --stats`` for a per-kernel table of one engine.
"""
from __future__ import annotations

import argparse
import collections
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tensorrt_dft_plugins_amd.engine import Engine  # noqa: E402
from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet  # noqa: E402


def build(export: str, cfg, x):
    torch.manual_seed(1234)
    m = AFNONet(cfg, backend=export).cuda().eval()
    t0 = time.time()
    e = Engine.build(m, (x,), device=x.device)
    print(f"[diff] {export}: built in {time.time() - t0:.1f}s, {len(e.graph.nodes)} nodes", file=sys.stderr, flush=True)
    del m
    torch.cuda.empty_cache()
    return e


def ops(e):
    return [n[4] for n in e.graph.nodes]


def time_ms(e, iters):
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        e.enqueue()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--export", default="both", choices=["both", "contrib", "amd"])
    a = ap.parse_args()
    cfg = AFNOConfig(depth=a.depth)
    torch.manual_seed(0)
    x = torch.randn(a.batch, cfg.in_chans, *cfg.img_size, device="cuda")
    which = ["contrib", "amd"] if a.export == "both" else [a.export]
    engs = {w: build(w, cfg, x) for w in which}
    for w, e in engs.items():
        e.static_inputs[0].copy_(x)
        print(f"{w}: {len(ops(e))} nodes: " + " ".join(ops(e)), flush=True)
    if len(engs) == 2:
        ca, cb = collections.Counter(ops(engs["contrib"])), collections.Counter(ops(engs["amd"]))
        print("op counts differing (contrib vs amd):", {k: (ca[k], cb[k]) for k in sorted(set(ca) | set(cb)) if ca[k] != cb[k]},
              flush=True)
        ya, yb = engs["contrib"].infer(x)[0], engs["amd"].infer(x)[0]
        print(f"rel-L2 contrib vs amd engine output: {float((ya - yb).norm() / yb.norm()):.3e}", flush=True)
    for w, e in engs.items():
        time_ms(e, 2)
    res = collections.defaultdict(list)
    for r in range(a.rounds):
        for w, e in engs.items():
            res[w].append(time_ms(e, a.iters))
    for w in engs:
        v = sorted(res[w])
        print(f"{w}: ms/step median {v[len(v) // 2]:.3f} min {v[0]:.3f} all {[round(t, 3) for t in res[w]]}", flush=True)


if __name__ == "__main__":
    main()
