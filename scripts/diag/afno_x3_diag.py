"""Diagnose the bf16x3 AFNO spectral kernel error: per-component comparisons."""
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
B, H, KM, C, nb = int(os.environ.get('DB', 2)), 90, int(os.environ.get('DKM', 46)), 768, 8
bs = C // nb
xw = torch.randn(B, H, KM, C, 2)
w1, w2 = 0.05 * torch.randn(2, nb, bs, bs), 0.05 * torch.randn(2, nb, bs, bs)
b1, b2 = 0.05 * torch.randn(2, nb, bs), 0.05 * torch.randn(2, nb, bs)
w1t = S._real_block(w1).transpose(1, 2).contiguous(); w2t = S._real_block(w2).transpose(1, 2).contiguous()
b1p, b2p = torch.cat([b1[0], b1[1]], 1), torch.cat([b2[0], b2[1]], 1)
ref = ops.afno_spectral(xw, w1t, w2t, b1p, b2p, 0.01)
w1s, w2s = S.split_bf16(w1t.to(dev)), S.split_bf16(w2t.to(dev))
ref_split = ops.afno_spectral(xw, w1s.cpu(), w2s.cpu(), b1p, b2p, 0.01)
out = ops.afno_spectral(xw.to(dev), w1s, w2s, b1p.to(dev), b2p.to(dev), 0.01).cpu()
outb = ops.afno_spectral(xw.to(dev), w1t.to(dev).bfloat16(), w2t.to(dev).bfloat16(), b1p.to(dev), b2p.to(dev), 0.01).cpu()
print("x3 vs ref", rel(out, ref), "ref_split vs ref", rel(ref_split, ref), "bf16kern vs ref", rel(outb, ref), "x3 vs bf16kern", rel(out, outb))
d = (out - ref).double()
print("err per h (first 12):", [round((d[:, h].norm() / ref[:, h].double().norm()).item(), 6) for h in range(12)])
print("err per block:", [round((d[..., i*96:(i+1)*96, :].norm() / ref[..., i*96:(i+1)*96, :].double().norm()).item(), 6) for i in range(8)])
print("err per kw:", [round((d[:, :, k].norm() / ref[:, :, k].double().norm()).item(), 6) for k in range(KM)])
print("err per b:", [round((d[b].norm() / ref[b].double().norm()).item(), 6) for b in range(B)])
p1, p2, p3, p4 = S.pack_afno_weights(w1.to(dev), b1.to(dev), w2.to(dev), b2.to(dev), split=True)
print("pack vs direct split equal:", torch.equal(p1.cpu(), w1s.cpu()), torch.equal(p2.cpu(), w2s.cpu()), torch.equal(p3.cpu(), b1p), torch.equal(p4.cpu(), b2p))
out2 = ops.afno_spectral(xw.to(dev), p1, p2, p3, p4, 0.01).cpu()
print("x3(pack) vs ref", rel(out2, ref))
# identity weights: FFT-only path
I = torch.zeros(2, nb, bs, bs); I[0] = torch.eye(bs)
z = torch.zeros(2, nb, bs)
wi = S._real_block(I).transpose(1, 2).contiguous()
xpos = xw.abs()
refi = ops.afno_spectral(xpos, wi, wi, z.reshape(nb, -1).repeat(1, 1)[:, :0].new_zeros(nb, 2*bs), torch.zeros(nb, 2*bs), 0.0)
wis = S.split_bf16(wi.to(dev))
outi = ops.afno_spectral(xpos.to(dev), wis, wis, torch.zeros(nb, 2*bs, device=dev), torch.zeros(nb, 2*bs, device=dev), 0.0).cpu()
print("identity-weights x3 vs ref", rel(outi, refi))
