"""Which GELU does hipBLASLt's fused epilogue (torch._addmm_activation(use_gelu=True)) compute?
Compares against erf-GELU (nn.GELU(), FourCastNet) and tanh-GELU on fp32 and bf16 GEMMs."""
import json

import torch
import torch.nn.functional as F


def main():
    torch.manual_seed(0)
    res = {}
    for dt in (torch.float32, torch.bfloat16):
        x = (2 * torch.randn(4096, 768, device="cuda")).to(dt)
        w = (torch.randn(3072, 768, device="cuda") / 768 ** 0.5).to(dt)
        b = torch.zeros(3072, device="cuda", dtype=dt)
        fused = torch._addmm_activation(b, x, w.t(), use_gelu=True).float()
        pre = (x.float() @ w.float().t())
        e = F.gelu(pre)
        t = F.gelu(pre, approximate="tanh")
        res[str(dt)] = {"max_abs_vs_erf": (fused - e).abs().max().item(),
                        "max_abs_vs_tanh": (fused - t).abs().max().item(),
                        "erf_vs_tanh": (e - t).abs().max().item()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
