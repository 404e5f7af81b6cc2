"""Stage-wise check of the bf16x3 AFNO kernel at a co-resident grid (MI_DFT_AFNO_DBG=1/2)."""
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
nb, bs, H, C, B, KM = 8, 96, 90, 768, 2, 46
w1, w2 = 0.05 * torch.randn(2, nb, bs, bs), 0.05 * torch.randn(2, nb, bs, bs)
b1, b2 = 0.05 * torch.randn(2, nb, bs), 0.05 * torch.randn(2, nb, bs)
w1t = S._real_block(w1).transpose(1, 2).contiguous(); w2t = S._real_block(w2).transpose(1, 2).contiguous()
b1p, b2p = torch.cat([b1[0], b1[1]], 1), torch.cat([b2[0], b2[1]], 1)
w1s, w2s = S.split_bf16(w1t.to(dev)), S.split_bf16(w2t.to(dev))
xw = torch.randn(B, H, KM, C, 2)
X = torch.view_as_real(torch.fft.fft(torch.view_as_complex(xw), dim=1))  # [B,H,KM,C,2]
Xr = X.reshape(B, H, KM, nb, bs, 2)
A = torch.cat([Xr[..., 0], Xr[..., 1]], -1)
H1 = torch.relu(torch.einsum("...bk,bkn->...bn", A, w1t.transpose(1, 2)) + b1p)
H1c = torch.stack([H1[..., :bs], H1[..., bs:]], -1).reshape(B, H, KM, C, 2)
stage = int(os.environ["MI_DFT_AFNO_DBG"])
ref = X if stage in (1, 3) else H1c
for it in range(3):
    out = ops.afno_spectral(xw.to(dev), w1s, w2s, b1p.to(dev), b2p.to(dev), 0.01).cpu()
    d = (out - ref).double()
    bad = [(k, bl) for k in range(KM) for bl in range(nb) if (d[:, :, k, bl*bs:(bl+1)*bs].norm() / ref[:, :, k, bl*bs:(bl+1)*bs].double().norm()) > 1e-4]
    print(f"stage {stage} run {it}: rel {rel(out, ref):.3e} bad tiles {bad[:10]}", flush=True)
    if bad:
        k, bl = bad[0]
        for b in range(B):
            t = d[b, :, k, bl*bs:(bl+1)*bs].norm(dim=(-1,))  # [H, bs]
            rows = (t.norm(dim=1) > 1e-3 * ref[b, :, k, bl*bs:(bl+1)*bs].double().norm() / 10).nonzero().flatten().tolist()
            cols = (t.norm(dim=0) > 1e-3 * ref[b, :, k, bl*bs:(bl+1)*bs].double().norm() / 10).nonzero().flatten().tolist()
            print(f"   b={b} bad rows {rows[:40]} bad cols {cols[:40]}", flush=True)
