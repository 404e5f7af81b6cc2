"""Sweep FFT pass tilings (MI_DFT_LOGT_ROW / MI_DFT_LOGT_COL / MI_DFT_THREADS) for one
shape in one process (interleaved rounds) and print the time of each configuration.

Usage: python bench/tune_fft.py [--shape 720 1440] [--batch 1] [--op rfft2|irfft2]
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from bench.bench_fft import time_graph  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", type=int, nargs=2, default=[720, 1440])
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--op", default="rfft2")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--rows", default="0,1,2")
    ap.add_argument("--cols", default="0,1,2,3,4")
    ap.add_argument("--threads", default="64,128,256")
    a = ap.parse_args(argv)
    H, W = a.shape
    x = torch.randn(a.batch, H, W, device="cuda")
    y = tdp.contrib_rfft(x, signal_ndim=2)
    fn = (lambda: tdp.contrib_rfft(x, signal_ndim=2)) if a.op == "rfft2" else (lambda: tdp.contrib_irfft(y, signal_ndim=2))
    cfgs = list(itertools.product(a.rows.split(","), a.cols.split(","), a.threads.split(",")))
    res = {c: [] for c in cfgs}
    for _ in range(a.rounds):
        for c in cfgs:
            os.environ["MI_DFT_LOGT_ROW"], os.environ["MI_DFT_LOGT_COL"], os.environ["MI_DFT_THREADS"] = c
            res[c].append(time_graph(fn, 30))
    rows = sorted(((statistics.median(v), c) for c, v in res.items()))
    for t, c in rows[:15]:
        print(f"{a.op} row_logT={c[0]} col_logT={c[1]} threads={c[2]}: {t:.2f} us")
    print(json.dumps({"best": rows[0][1], "best_us": rows[0][0]}))


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import note_tuning_build

    note_tuning_build("MI_DFT_LOGT_ROW / MI_DFT_LOGT_COL / MI_DFT_THREADS")
    main()
