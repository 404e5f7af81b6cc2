"""MLP sub-block variants (FourCastNet fc1 768->3072 GELU, fc2 3072->768) at M = 32*16200 bf16."""
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

M, C, Hd = 32 * 16200, 768, 3072
dev = "cuda"
x = torch.randn(M, C, device=dev, dtype=torch.bfloat16)
r = torch.randn(M, C, device=dev, dtype=torch.bfloat16)
w1 = torch.randn(Hd, C, device=dev, dtype=torch.bfloat16) * 0.02
b1 = torch.randn(Hd, device=dev, dtype=torch.bfloat16) * 0.02
w2 = torch.randn(C, Hd, device=dev, dtype=torch.bfloat16) * 0.02
b2 = torch.randn(C, device=dev, dtype=torch.bfloat16) * 0.02


def t(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


ref = F.gelu(F.linear(x, w1, b1))
variants = {
    "linear+gelu": lambda: F.gelu(F.linear(x, w1, b1)),
    "linear+gelu_tanh": lambda: F.gelu(F.linear(x, w1, b1), approximate="tanh"),
    "addmm_act_gelu": lambda: torch._addmm_activation(b1, x, w1.t(), use_gelu=True),
    "linear_only": lambda: F.linear(x, w1, b1),
    "mm_nobias": lambda: torch.mm(x, w1.t()),
    "fc2_addmm_res": lambda: torch.addmm(r, ref, w2.t()),
    "fc2_mm": lambda: torch.mm(ref, w2.t()),
    "fc2_linear": lambda: F.linear(ref, w2, b2),
}
for k, f in variants.items():
    ms = t(f)
    print(f"{k:18s} {ms:8.3f} ms")
y = torch._addmm_activation(b1, x, w1.t(), use_gelu=True)
print("addmm_act vs erf gelu max abs diff", (y.float() - ref.float()).abs().max().item(),
      "vs tanh", (y.float() - F.gelu(F.linear(x, w1, b1), approximate="tanh").float()).abs().max().item())

# operand-layout variants (hipBLASLt picks different kernels per transpose case)
w1t = w1.t().contiguous()  # [C, Hd]
w2t = w2.t().contiguous()  # [Hd, C]
hid = ref
layout = {
    "fc1 x@W^T (TN)": lambda: torch.mm(x, w1.t()),
    "fc1 x@Wt (NN)": lambda: torch.mm(x, w1t),
    "fc1 (W x^T)^T": lambda: torch.mm(w1, x.t()),
    "fc2 h@W^T (TN)": lambda: torch.mm(hid, w2.t()),
    "fc2 h@Wt (NN)": lambda: torch.mm(hid, w2t),
    "fc2 (W h^T)^T": lambda: torch.mm(w2, hid.t()),
}
for k, f in layout.items():
    ms = t(f)
    print(f"{k:18s} {ms:8.3f} ms  {2 * M * C * Hd / ms / 1e9:7.1f} TFLOP/s")
