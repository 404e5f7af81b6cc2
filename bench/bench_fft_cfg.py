"""rfft2 / irfft2 720x1440 latency per column-pass tile config (MI_DFT_FIXED_CFG) and XCD-aware
tile order (MI_DFT_FFT_XCD), one process, interleaved.
(Tuning build only: the switches are read by a library built with -DAMD_DFT_TUNING=1, csrc/ops/tuning.h.)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from bench.bench_fft import time_graph  # noqa: E402

tdp.load_plugins()
x = torch.randn(1, 720, 1440, device="cuda")
y = tdp.contrib_rfft(x, signal_ndim=2)
cfgs = sys.argv[1:] or ["auto", "90,2", "90,4", "90,8", "45,4", "45,8", "45,16"]
res = {}
for _ in range(3):
    for cfg in cfgs:
        for xcd in ("0", "1"):
            os.environ["MI_DFT_FFT_XCD"] = xcd
            if cfg == "auto":
                os.environ.pop("MI_DFT_FIXED_CFG", None)
            else:
                os.environ["MI_DFT_FIXED_CFG"] = cfg
            f1 = lambda: tdp.contrib_rfft(x, signal_ndim=2)  # noqa: E731
            f2 = lambda: tdp.contrib_irfft(y, signal_ndim=2)  # noqa: E731
            f1(), f2()
            r = res.setdefault((cfg, xcd), {"rfft2": [], "irfft2": []})
            r["rfft2"].append(time_graph(f1, 50))
            r["irfft2"].append(time_graph(f2, 50))
for (cfg, xcd), r in res.items():
    print(f"cfg={cfg:6s} xcd={xcd}", json.dumps({k: round(min(v), 2) for k, v in r.items()}), flush=True)
