"""fc2 variants on the FourCastNet shape (M = 518400, 3072 -> 768, bf16): bias epilogue vs
in-place beta=1 accumulation into the residual stream (addmm_)."""
import torch
import torch.nn.functional as F

from bench_fft import time_graph

M, C, Hd = 32 * 16200, 768, 3072
h = torch.randn(M, Hd, device="cuda").to(torch.bfloat16)
x = torch.randn(M, C, device="cuda").to(torch.bfloat16)
w2 = (torch.randn(C, Hd, device="cuda") * 0.02).to(torch.bfloat16)
b2 = (torch.randn(C, device="cuda") * 0.02).to(torch.bfloat16)
x0 = x.clone()
res = {}
res["linear_bias"] = time_graph(lambda: F.linear(h, w2, b2), 5)
res["addmm_inplace"] = time_graph(lambda: x.addmm_(h, w2.t()), 5)
res["addmm_out"] = time_graph(lambda: torch.addmm(x0, h, w2.t()), 5)
xr = x0.clone()
xr.addmm_(h, w2.t())
ref = x0.float() + h.float() @ w2.float().t()
print({k: round(v, 1) for k, v in res.items()}, "err", (xr.float() - ref).abs().max().item())
