"""HBM streaming calibration on the tensor sizes of the spectral benchmarks: time of a plain
read (sum), copy and fill with PyTorch's own kernels, to put kernel times in context
(small transfers do not reach the 8 TB/s peak; this measures what they do reach).

Usage: python bench/membw.py [--mb 41.5 83 166 ...]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench.bench_fft import time_graph  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, nargs="+", default=[10.4, 41.5, 83.0, 332.0, 1327.0])
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args(argv)
    res = []
    for mb in a.mb:
        n = int(mb * 1e6 / 4)
        x = torch.randn(n, device="cuda")
        y = torch.empty_like(x)
        r = {"MB": mb}
        r["read_sum_us"] = time_graph(lambda: x.sum(), a.iters)
        r["copy_us"] = time_graph(lambda: y.copy_(x), a.iters)
        r["fill_us"] = time_graph(lambda: y.fill_(1.0), a.iters)
        r["read_TBps"] = mb * 1e6 / (r["read_sum_us"] * 1e-6) / 1e12
        r["copy_TBps(r+w)"] = 2 * mb * 1e6 / (r["copy_us"] * 1e-6) / 1e12
        print(json.dumps(r), flush=True)
        res.append(r)
    return res


if __name__ == "__main__":
    main()
