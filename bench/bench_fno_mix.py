"""FNO block (BASELINE config 3 shape: 20 ch, 720x1440, modes 32x32) at batch 1 / 8 / 32 with both
mode-mixing paths of the amd backend: 1 = the mixing gather inside the pruned inverse H transform,
2 = batched per-mode GEMMs on MFMA (csrc/spectral/fno_mix.hip) + the pruned inverse C2C; and the
default (0, by batch size).  hipGraph-replay medians, interleaved rounds in one process.

Usage: python bench/bench_fno_mix.py [--batches 1 8 32] [--rounds 5] [--dtype bf16 fp32]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from bench.bench_fft import time_graph  # noqa: E402
from tensorrt_dft_plugins_amd.models.fno import FNOBlock  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, nargs="+", default=[1, 8, 32])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--dtype", nargs="+", default=["bf16", "fp32"])
    a = ap.parse_args(argv)
    tdp.load_plugins()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    blk = FNOBlock(20, 32, 32, backend="amd").to(dev).eval()
    for tag in a.dtype:
        dt = torch.bfloat16 if tag == "bf16" else torch.float32
        for B in a.batches:
            x = torch.randn(B, 20, 720, 1440, device=dev).to(dt)
            samples = {p: [] for p in (0, 1, 2)}
            with torch.no_grad():
                outs = {}
                for p in (1, 2):
                    blk.mix_path = p
                    outs[p] = blk(x).float()
                diff = float((outs[1] - outs[2]).norm() / outs[1].norm())
                for _ in range(a.rounds):
                    for p in (0, 1, 2):
                        blk.mix_path = p
                        samples[p].append(time_graph(lambda: blk(x), a.iters))
            r = {"dtype": tag, "batch": B, "rel_diff_paths": diff}
            for p, name in ((0, "default"), (1, "gather"), (2, "mfma")):
                med = statistics.median(samples[p])
                r[f"{name}_us"] = round(med, 2)
                r[f"{name}_us_per_sample"] = round(med / B, 2)
            print(json.dumps(r), flush=True)
            del x, outs
            torch.cuda.empty_cache()
    blk.mix_path = 0


if __name__ == "__main__":
    main()
