"""dftw_r2c (truncated W-DFT on MFMA, 1440 -> 32 modes, bf16 rows) timed at row counts around the FNO
layer's 14400 (= 900 sixteen-row workgroups, 3.5 per CU): is the one-round grid's per-CU imbalance visible?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402


def graph_us(fn, iters=20, rounds=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000.0 / iters)
    return sorted(ts)[len(ts) // 2]


tdp.load_plugins()
for rows in (12288, 14400, 16384, 8192, 4096):
    x = torch.randn(rows, 1440, device="cuda").to(torch.bfloat16)
    us = graph_us(lambda: torch.ops.amd_dft.dftw_r2c(x, 32, 1.0))
    print(f"dftw_r2c rows {rows:6d} ({rows // 16:5d} workgroups): {us:7.2f} us  {us / rows * 1e3:6.3f} ns/row", flush=True)
