"""Run the FourCastNet MLP GEMMs with a forced TunableOp solution table (lookup only), for
rocprofv3 kernel-name / interference checks.  python scripts/gemm_forced.py TABLE.csv [iters]"""
import sys

import torch
import torch.cuda.tunable as tunable

table = sys.argv[1]
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
tunable.enable(True)
tunable.tuning_enable(False)
tunable.set_filename("/tmp/unused_tunable.csv")
assert tunable.read_file(table), "table rejected"
M, C, Hd = 32 * 16200, 768, 3072
x = torch.randn(M, C, device="cuda").to(torch.bfloat16)
h = torch.randn(M, Hd, device="cuda").to(torch.bfloat16)
w1 = (torch.randn(Hd, C, device="cuda") * 0.02).to(torch.bfloat16)
w2 = (torch.randn(C, Hd, device="cuda") * 0.02).to(torch.bfloat16)
b1 = (torch.randn(Hd, device="cuda") * 0.02).to(torch.bfloat16)
for _ in range(iters):
    torch._addmm_activation(b1, x, w1.t(), use_gelu=True)
    x.addmm_(h, w2.t())
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    torch._addmm_activation(b1, x, w1.t(), use_gelu=True)
t1 = torch.cuda.Event(enable_timing=True)
t1.record()
for _ in range(5):
    x.addmm_(h, w2.t())
e1.record()
torch.cuda.synchronize()
print(f"fc1 {e0.elapsed_time(t1) / 5:.3f} ms  fc2 {t1.elapsed_time(e1) / 5:.3f} ms", flush=True)
