"""Large-grid determinism + accuracy screen of every native kernel family (workgroups co-resident
on the CUs): each op runs 3x on the same input; outputs must be bit-identical and match the CPU
(ATen fp32) implementation of the same op.  A kernel that is exact on small grids but not here
has a cross-wave race or a miscompile (see csrc/spectral/afno_spectral.hip header).
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from tensorrt_dft_plugins_amd.models.fno import FNOBlock  # noqa: E402
from tensorrt_dft_plugins_amd.ops import spectral as S  # noqa: E402

tdp.load_plugins()
ops = torch.ops.amd_dft
dev = "cuda"
bad = []


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm()).item()


def check(name, fn_gpu, ref, tol):
    outs = [fn_gpu() for _ in range(3)]
    outs = [o.cpu() if isinstance(o, torch.Tensor) else o[0].cpu() for o in outs]
    det = all(torch.equal(outs[0], o) for o in outs[1:])
    err = [rel(o.float(), ref.float()) for o in outs]
    ok = det and max(err) < tol
    if not ok:
        bad.append(name)
    print(f"{'OK ' if ok else 'BAD'} {name:40s} det={det} err={[f'{e:.2e}' for e in err]} tol={tol}", flush=True)


torch.manual_seed(0)
# rfft2 / irfft2 720x1440 batch 8
x = torch.randn(8, 720, 1440)
ref = ops.Rfft(x, 0, 1, 2)
xd = x.to(dev)
check("Rfft 8x720x1440", lambda: ops.Rfft(xd, 0, 1, 2), ref, 1e-5)
check("Irfft 8x720x1440", lambda: ops.Irfft(ref.to(dev), 0, 1, 2), ops.Irfft(ref, 0, 1, 2), 1e-5)
# AFNO W transforms, bf16 and fp32, B=8
B, H, W, C = 8, 90, 180, 768
xa = torch.randn(B, H, W, C)
g, be, pre = torch.randn(C) * 0.3 + 1, torch.randn(C) * 0.1, torch.randn(C) * 0.2
scale = 1.0 / math.sqrt(H * W)
for dt, tol in ((torch.float32, 2e-6), (torch.bfloat16, 1e-2)):
    xx = xa.to(dt)
    st = ops.ln_stats(xx, pre, 1e-6)
    r1 = ops.r2c_ln(xx, 2, scale, 46, st, g, be, pre, dt)
    xd = xx.to(dev)
    std = ops.ln_stats(xd, pre.to(dev), 1e-6)
    check(f"ln_stats {dt}", lambda: ops.ln_stats(xd, pre.to(dev), 1e-6), st, 1e-5)
    check(f"r2c_ln {dt}", lambda: ops.r2c_ln(xd, 2, scale, 46, std, g.to(dev), be.to(dev), pre.to(dev), dt), r1, tol)
    X = torch.randn(B, H, 46, C, 2).to(dt)
    r2 = ops.c2r_ln_add(X, 2, W, scale, xx, st, g, be, pre)
    Xd = X.to(dev)
    check(f"c2r_ln_add {dt}", lambda: ops.c2r_ln_add(Xd, 2, W, scale, xd, std, g.to(dev), be.to(dev), pre.to(dev)), r2, tol)
# layer norms
xl = torch.randn(100000, 768)
gl, bl = torch.randn(768), torch.randn(768)
check("layer_norm fp32", lambda: ops.layer_norm(xl.to(dev), gl.to(dev), bl.to(dev), 1e-6, None)[0],
      ops.layer_norm(xl, gl, bl, 1e-6, None)[0], 1e-5)
check("layer_norm_split", lambda: ops.layer_norm_split(xl.to(dev), gl.to(dev), bl.to(dev), 1e-6, None),
      ops.layer_norm_split(xl, gl, bl, 1e-6, None), 1e-2)
xlb = xl.to(torch.bfloat16)
check("layer_norm bf16", lambda: ops.layer_norm(xlb.to(dev), gl.to(dev).bfloat16(), bl.to(dev).bfloat16(), 1e-6, None)[0],
      ops.layer_norm(xlb, gl.bfloat16(), bl.bfloat16(), 1e-6, None)[0], 1e-2)
# GEMMs (bf16 and bf16x3), M = 65536 rows (768 workgroups)
M = 65536
xg = torch.randn(M, 768)
wg = torch.randn(3072, 768) * 0.03
bg = torch.randn(3072) * 0.1
check("linear bf16 fc1+gelu", lambda: ops.linear(xg.to(dev).bfloat16(), wg.to(dev).bfloat16(), bg.to(dev), 1, None),
      torch.nn.functional.gelu(xg @ wg.t() + bg), 1e-2)
check("linear3 fc1+gelu", lambda: ops.linear3(ops.split_bf16(xg.to(dev)), ops.split_bf16(wg.to(dev)), bg.to(dev), 1, None, False),
      torch.nn.functional.gelu(xg @ wg.t() + bg), 2e-5)
# FNO block (dftw_r2c, c2c_axis, fno_mix_c2c, fno_c2r_pw), batch 4, 720x1440
blk_t = FNOBlock(20, 32, 32, backend="torch").eval()
blk_a = FNOBlock(20, 32, 32, backend="amd").to(dev).eval()
blk_a.load_state_dict(blk_t.state_dict())
xf = torch.randn(4, 20, 720, 1440)
with torch.no_grad():
    rf = blk_t(xf)
    check("FNO block fp32", lambda: blk_a(xf.to(dev)), rf, 1e-4)
    check("FNO block bf16", lambda: blk_a(xf.to(dev).bfloat16()), rf, 2e-2)
# AFNO spectral (both variants) at the bench grid
nb, bs = 8, 96
w1, w2 = 0.05 * torch.randn(2, nb, bs, bs), 0.05 * torch.randn(2, nb, bs, bs)
b1, b2 = 0.05 * torch.randn(2, nb, bs), 0.05 * torch.randn(2, nb, bs)
w1t = S._real_block(w1).transpose(1, 2).contiguous()
w2t = S._real_block(w2).transpose(1, 2).contiguous()
b1p, b2p = torch.cat([b1[0], b1[1]], 1), torch.cat([b2[0], b2[1]], 1)
xw = torch.randn(16, H, 46, C, 2)
ra = ops.afno_spectral(xw, w1t, w2t, b1p, b2p, 0.01)
pk3 = S.pack_afno_weights(w1.to(dev), b1.to(dev), w2.to(dev), b2.to(dev), split=True)
pkb = S.pack_afno_weights(w1.to(dev), b1.to(dev), w2.to(dev), b2.to(dev), split=False)
check("afno_spectral x3", lambda: ops.afno_spectral(xw.to(dev), *pk3, 0.01), ra, 1e-5)
check("afno_spectral bf16", lambda: ops.afno_spectral(xw.to(dev).bfloat16(), *pkb, 0.01), ra, 1e-2)
print("BAD:", bad)
sys.exit(1 if bad else 0)
