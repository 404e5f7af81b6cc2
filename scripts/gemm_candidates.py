"""List hipBLASLt candidate solutions (TunableOp, verbose) for the FourCastNet MLP GEMMs as the
model issues them: fc1 = _addmm_activation(GELU) and fc2 = in-place addmm_ (beta = 1)."""
import os
import sys

import torch

M, C, Hd = 32 * 16200, 768, 3072
import torch.cuda.tunable as tunable  # noqa: E402

tunable.enable(True)
tunable.tuning_enable(True)
tunable.set_max_tuning_duration(int(os.environ.get("TUNE_MS", "40")))
tunable.set_filename(f"/tmp/tunable_{os.getpid()}.csv")
x = torch.randn(M, C, device="cuda").to(torch.bfloat16)
h = torch.randn(M, Hd, device="cuda").to(torch.bfloat16)
w1 = (torch.randn(Hd, C, device="cuda") * 0.02).to(torch.bfloat16)
w2 = (torch.randn(C, Hd, device="cuda") * 0.02).to(torch.bfloat16)
b1 = (torch.randn(Hd, device="cuda") * 0.02).to(torch.bfloat16)
torch._addmm_activation(b1, x, w1.t(), use_gelu=True)
x.addmm_(h, w2.t())
torch.cuda.synchronize()
for r in tunable.get_results():
    print("RESULT", r, flush=True)
