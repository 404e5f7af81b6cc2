"""A/B the specialised column-pass configurations (MI_DFT_FIXED_CFG) and the generic kernel
for rfft2/irfft2 720x1440 (interleaved rounds, hipGraph timing).
(Tuning build only: the switches are read by a library built with -DAMD_DFT_TUNING=1, csrc/ops/tuning.h.)"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from bench.bench_fft import time_graph  # noqa: E402

B = int(os.environ.get("TUNE_B", "1"))
x = torch.randn(B, 720, 1440, device="cuda")
y = tdp.contrib_rfft(x, signal_ndim=2)
ops = {"rfft2": lambda: tdp.contrib_rfft(x, signal_ndim=2), "irfft2": lambda: tdp.contrib_irfft(y, signal_ndim=2)}
variants = {"auto": {}, "generic": {"MI_DFT_FIXED": "0"}}
for c in ["90,4", "90,2", "45,8", "45,4"]:
    variants["col" + c] = {"MI_DFT_FIXED_CFG": c}
res = {}
for _ in range(7):
    for vn, env in variants.items():
        for k in ("MI_DFT_FIXED", "MI_DFT_FIXED_CFG"):
            os.environ.pop(k, None)
        os.environ.update(env)
        for on, f in ops.items():
            res.setdefault((on, vn), []).append(time_graph(f, 30))
for (on, vn), v in sorted(res.items()):
    print(f"B={B} {on:7s} {vn:10s} {statistics.median(v):8.2f} us")
