"""AFNO spectral kernels: error vs grid size, repeat determinism (LDS pad via MI_DFT_AFNO_LDS_PAD)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import tensorrt_dft_plugins_amd as tdp
from tensorrt_dft_plugins_amd.ops import spectral as S
tdp.load_plugins()
ops = torch.ops.amd_dft
dev = "cuda"
def rel(a, b): a, b = a.double().cpu(), b.double().cpu(); return ((a - b).norm() / b.norm()).item()
torch.manual_seed(4)
nb, bs, H, C = 8, 96, 90, 768
w1, w2 = 0.05 * torch.randn(2, nb, bs, bs), 0.05 * torch.randn(2, nb, bs, bs)
b1, b2 = 0.05 * torch.randn(2, nb, bs), 0.05 * torch.randn(2, nb, bs)
w1t = S._real_block(w1).transpose(1, 2).contiguous(); w2t = S._real_block(w2).transpose(1, 2).contiguous()
b1p, b2p = torch.cat([b1[0], b1[1]], 1), torch.cat([b2[0], b2[1]], 1)
w1s, w2s = S.split_bf16(w1t.to(dev)), S.split_bf16(w2t.to(dev))
w1b, w2b = w1t.to(dev).bfloat16(), w2t.to(dev).bfloat16()
for B, KM in ((1, 4), (1, 16), (1, 46), (2, 46), (8, 46)):
    xw = torch.randn(B, H, KM, C, 2)
    ref = ops.afno_spectral(xw, w1t, w2t, b1p, b2p, 0.01)
    xd = xw.to(dev)
    o = [ops.afno_spectral(xd, w1s, w2s, b1p.to(dev), b2p.to(dev), 0.01).cpu() for _ in range(3)]
    ob = [ops.afno_spectral(xd, w1b, w2b, b1p.to(dev), b2p.to(dev), 0.01).cpu() for _ in range(3)]
    print(f"B={B} KM={KM}: x3 err {[round(rel(t, ref), 7) for t in o]} det {torch.equal(o[0], o[1]) and torch.equal(o[1], o[2])} | "
          f"bf16 err {[round(rel(t, ref), 5) for t in ob]} det {torch.equal(ob[0], ob[1]) and torch.equal(ob[1], ob[2])}", flush=True)
