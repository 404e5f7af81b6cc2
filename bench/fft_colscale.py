"""Column-pass scaling probe: C2C length-720 FFT along H over 721 / 361 / 181 / 91 columns
(graph-timed).  Time proportional to the column count = SIMD-throughput bound; flat = latency
bound (what decides whether packing two columns per thread can pay)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from bench.bench_fft import time_graph  # noqa: E402
from tensorrt_dft_plugins_amd.ops import dft as D  # noqa: E402

tdp.load_plugins()
for ncol in (721, 361, 181, 91):
    yc = torch.randn(1, 720, ncol, dtype=torch.complex64, device="cuda")
    f = lambda: D.fft(yc, dim=-2, return_real=True)  # noqa: E731
    f()
    print(f"cols={ncol:4d} {min(time_graph(f, 50) for _ in range(5)):7.2f} us", flush=True)
x = torch.randn(1, 720, 1440, device="cuda")
for nrow in (720, 360, 180, 90):
    xr = x[:, :nrow].contiguous()
    f = lambda: D.rfft(xr, dim=-1, return_real=True)  # noqa: E731
    f()
    print(f"rows={nrow:4d} {min(time_graph(f, 50) for _ in range(5)):7.2f} us", flush=True)
