"""Single-GPU proxy for the multi-GPU all-gather's CU footprint: while the captured FourCastNet
step replays, N long-running single-workgroup spin kernels (torch.cuda._sleep, one per side
stream, like one RCCL channel each) occupy N CUs.  Reports ms/step with and without them, to see
how much a concurrent collective costs the stream-K hipBLASLt GEMMs and the hand kernels.

  python scripts/interference_probe.py [--spinners 0 16 32] [--steps 4]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from tensorrt_dft_plugins_amd.engine.capture import CapturedModule  # noqa: E402
from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--spinners", type=int, nargs="+", default=[0, 8, 32])
ap.add_argument("--steps", type=int, default=4)
ap.add_argument("--cycles", type=int, default=100_000_000, help="spin length per kernel (GPU clock cycles)")
ap.add_argument("--table", default=None, help="TunableOp solution table (lookup only)")
a = ap.parse_args()
tdp.load_plugins()
if a.table:
    import torch.cuda.tunable as tunable

    tunable.enable(True)
    tunable.tuning_enable(False)
    tunable.set_filename("/tmp/unused_tunable.csv")
    assert tunable.read_file(a.table)
torch.manual_seed(0)
model = AFNONet(AFNOConfig(), backend="amd").cuda().to(torch.bfloat16).eval()
x = torch.randn(32, 20, 720, 1440, device="cuda").to(torch.bfloat16)
cap = CapturedModule(model, [x])
side = [torch.cuda.Stream() for _ in range(max(a.spinners))]
for n in a.spinners:
    cap.replay()
    torch.cuda.synchronize()
    for s in side[:n]:
        with torch.cuda.stream(s):
            torch.cuda._sleep(a.cycles)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        cap.replay()
    torch.cuda.synchronize(torch.cuda.current_device()) if n == 0 else torch.cuda.current_stream().synchronize()
    dt = (time.perf_counter() - t0) * 1000 / a.steps
    torch.cuda.synchronize()
    print(f"spinners={n:3d}  {dt:8.2f} ms/step", flush=True)
