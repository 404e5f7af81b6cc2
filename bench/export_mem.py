"""Peak device memory of the headline engine build (FourCastNet fp32, batch 32, depth 12, contrib export ->
optimizer -> engine) and of the export trace alone: the per-rank footprint of bench.py's build phase."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from tensorrt_dft_plugins_amd.engine import Engine  # noqa: E402
from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet  # noqa: E402
from tensorrt_dft_plugins_amd.onnx import exporter  # noqa: E402

tdp.load_plugins()
torch.manual_seed(0)
cfg = AFNOConfig()
m = AFNONet(cfg, backend="contrib").cuda().eval()
x = torch.randn(32, cfg.in_chans, *cfg.img_size, device="cuda")
gb = 1024 ** 3
base = torch.cuda.memory_allocated() / gb
torch.cuda.reset_peak_memory_stats()
t0 = time.perf_counter()
onnx_bytes = exporter.export(m, (x,))
print(f"export trace: {time.perf_counter() - t0:.1f} s, peak {torch.cuda.max_memory_allocated() / gb:.1f} GiB "
      f"(model + input {base:.1f} GiB)", flush=True)
torch.cuda.reset_peak_memory_stats()
t0 = time.perf_counter()
eng = Engine.build(onnx_bytes, shapes=[list(x.shape)], device=torch.device("cuda"), use_graph=True)
print(f"engine build (optimizer + capture): {time.perf_counter() - t0:.1f} s, peak "
      f"{torch.cuda.max_memory_allocated() / gb:.1f} GiB, optimizer {eng.header.extra.get('optimizer', {}).get('applied')}",
      flush=True)
