"""rfft2/irfft2 720x1440 fp32 broken into their passes (rows R2C, columns C2C, rows C2R), each
timed alone in a hipGraph, under the MI_DFT_FFT_ABLATE timing ablations (0 = full kernel,
2 = no twiddles, 6 = no twiddles and no butterflies: the kernels' data movement alone).
Compare with bench/fft_floor.hip (pure access-pattern floors)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from bench.bench_fft import time_graph  # noqa: E402
from tensorrt_dft_plugins_amd.ops import dft as D  # noqa: E402

tdp.load_plugins()
x = torch.randn(1, 720, 1440, device="cuda")
y = tdp.contrib_rfft(x, signal_ndim=2)          # [1, 720, 721, 2]
yc = torch.view_as_complex(y)
ops = {
    "rfft2": lambda: tdp.contrib_rfft(x, signal_ndim=2),
    "irfft2": lambda: tdp.contrib_irfft(y, signal_ndim=2),
    "rows_r2c": lambda: D.rfft(x, dim=-1, return_real=True),
    "cols_c2c": lambda: D.fft(yc, dim=-2, return_real=True),
    "rows_c2r": lambda: D.irfft(yc, n=1440, dim=-1),
}
# each argument: one environment setting, e.g. "MI_DFT_FFT_ABLATE=6" or
# "MI_DFT_FIXED_CFG=128,1;MI_DFT_FFT_XCD=1" (';'-separated)
specs = sys.argv[1:] or ["MI_DFT_FFT_ABLATE=0", "MI_DFT_FFT_ABLATE=2", "MI_DFT_FFT_ABLATE=6"]
res = {}
for _ in range(3):
    for spec in specs:
        kv = dict(e.split("=", 1) for e in spec.split(";") if e)
        os.environ.update(kv)
        for k, f in ops.items():
            f()
            res.setdefault((k, spec), []).append(time_graph(f, 50))
        for e in kv:
            os.environ.pop(e)
for (k, spec), v in sorted(res.items()):
    print(f"{k:10s} {spec:50s} {min(v):7.2f} us", flush=True)
