"""Timing-only ablations of the FFT pass kernels (MI_DFT_ABLATE), interleaved rounds."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from bench.bench_fft import time_graph  # noqa: E402

x = torch.randn(1, 720, 1440, device="cuda")
y = tdp.contrib_rfft(x, signal_ndim=2)
ops = {"rfft2": lambda: tdp.contrib_rfft(x, signal_ndim=2), "irfft2": lambda: tdp.contrib_irfft(y, signal_ndim=2),
       "rfft_rows": lambda: tdp.contrib_rfft(x, signal_ndim=1),
       "copy": lambda: y.clone()}
modes = ["", "nopass", "notw", "io"]
res = {}
for _ in range(5):
    for m in modes:
        os.environ["MI_DFT_ABLATE"] = m
        for k, f in ops.items():
            res.setdefault((k, m), []).append(time_graph(f, 30))
for (k, m), v in sorted(res.items()):
    print(f"{k:10s} {m or 'full':8s} {statistics.median(v):8.2f} us")
