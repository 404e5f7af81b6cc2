"""LayerNorm-fused AFNO W-transforms (ln_stats, r2c_ln, c2r_ln_add) and the fused block.

CPU tier: op semantics against plain torch (LayerNorm + torch.fft).  GPU tier: the HIP kernels
(specialised L=180 channel-last pair kernels) against the fp32/fp64 torch reference.
"""
import math

import pytest
import torch
import torch.nn.functional as F

ops = torch.ops.amd_dft


def rel_l2(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm()).item()


def _ln_ref(x, pre, g, b, eps):
    xp = x.double() + (0 if pre is None else pre.double())
    return xp, F.layer_norm(xp, (x.shape[-1],), g.double(), b.double(), eps)


def _inputs(B=2, H=6, W=12, C=16, dtype=torch.float32, device="cpu", seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, H, W, C, generator=g)
    pre = 0.3 * torch.randn(C, generator=g)
    gam = 1 + 0.1 * torch.randn(C, generator=g)
    bet = 0.1 * torch.randn(C, generator=g)
    return [t.to(device) for t in (x.to(dtype), pre, gam, bet)]


@pytest.mark.parametrize("with_pre", [False, True])
def test_ln_stats_cpu(with_pre):
    x, pre, _, _ = _inputs()
    p = pre if with_pre else None
    st = ops.ln_stats(x, p, 1e-6)
    xp = x.double() + (0 if p is None else p.double())
    var, mean = torch.var_mean(xp.reshape(-1, x.shape[-1]), dim=1, correction=0)
    assert st.shape == (x.numel() // x.shape[-1], 2)
    torch.testing.assert_close(st[:, 0].double(), mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(st[:, 1].double(), torch.rsqrt(var + 1e-6), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("with_pre", [False, True])
def test_r2c_ln_cpu_semantics(with_pre):
    x, pre, g, b = _inputs()
    p = pre if with_pre else None
    st = ops.ln_stats(x, p, 1e-6)
    km, scale = 4, 0.25
    out = ops.r2c_ln(x, 2, scale, km, st, g, b, p)
    _, h = _ln_ref(x, p, g, b, 1e-6)
    ref = torch.view_as_real(torch.fft.rfft(h, dim=2)[:, :, :km] * scale)
    assert out.shape == ref.shape
    assert rel_l2(out, ref) < 1e-5


@pytest.mark.parametrize("with_pre", [False, True])
def test_c2r_ln_add_cpu_semantics(with_pre):
    x, pre, g, b = _inputs(seed=1)
    p = pre if with_pre else None
    st = ops.ln_stats(x, p, 1e-6)
    km, W = 5, x.shape[2]
    X = torch.randn(2, 6, km, 16, 2)
    out = ops.c2r_ln_add(X, 2, W, 0.5, x, st, g, b, p)
    full = torch.zeros(2, 6, W // 2 + 1, 16, dtype=torch.complex128)
    full[:, :, :km] = torch.view_as_complex(X.double())
    xp, h = _ln_ref(x, p, g, b, 1e-6)
    ref = 0.5 * torch.fft.irfft(full, n=W, dim=2, norm="forward") + xp + h
    assert rel_l2(out, ref) < 1e-5


def test_ln_ops_meta_shapes():
    x = torch.empty(2, 6, 12, 16, device="meta")
    st = ops.ln_stats(x, None, 1e-6)
    assert st.shape == (144, 2)
    g = torch.empty(16, device="meta")
    X = ops.r2c_ln(x, 2, 1.0, 4, st, g, g, None)
    assert X.shape == (2, 6, 4, 16, 2)
    assert ops.c2r_ln_add(X, 2, 12, 1.0, x, st, g, g, None).shape == x.shape


def test_fused_block_matches_unfused_cpu_math():
    """afno_block_fused's data flow (stats -> LN-on-load R2C -> spectral -> C2R + both skips ->
    LN2 -> MLP accumulated into the stream, fc2 bias carried) equals the FourCastNet block."""
    from tensorrt_dft_plugins_amd.models import AFNOConfig
    from tensorrt_dft_plugins_amd.models.afno import Block

    torch.manual_seed(0)
    cfg = AFNOConfig(img_size=(48, 96), in_chans=4, out_chans=4, embed_dim=64, depth=1, num_blocks=4)
    blk = Block(cfg, backend="torch").eval()
    with torch.no_grad():
        blk.norm1.weight.normal_(1, 0.1)
        blk.norm1.bias.normal_(0, 0.1)
    x = torch.randn(2, cfg.h, cfg.w, cfg.embed_dim)
    pre = 0.1 * torch.randn(cfg.embed_dim)
    with torch.no_grad():
        ref = blk(x + pre)
        # the same data flow with the native CPU ops
        st = ops.ln_stats(x, pre, blk.norm1.eps)
        H, W = cfg.h, cfg.w
        scale = 1 / math.sqrt(H * W)
        from tensorrt_dft_plugins_amd.models.afno import kept_window

        r0, r1, km = kept_window(H, W, cfg.hard_thresholding_fraction)
        xw = ops.r2c_ln(x, 2, scale, km, st, blk.norm1.weight, blk.norm1.bias, pre)
        # H-direction filter on the W half spectrum (reference math on the kept modes)
        f = blk.filter
        h = F.layer_norm(x + pre, (cfg.embed_dim,), blk.norm1.weight, blk.norm1.bias, blk.norm1.eps)
        filt = f(h) - h  # filter output without its own bias (input) skip
        Yw = torch.fft.rfft(filt.double(), dim=2, norm="forward")[:, :, :km]
        x1 = ops.c2r_ln_add(torch.view_as_real(Yw).float().contiguous(), 2, W, 1.0, x, st, blk.norm1.weight,
                            blk.norm1.bias, pre)
        yn = blk.norm2(x1)
        out = x1 + blk.mlp(yn)
    assert xw.shape == (2, H, km, cfg.embed_dim, 2)
    assert rel_l2(out, ref) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("with_pre", [False, True])
def test_ln_fused_kernels_gpu(device, with_pre, recwarn):
    """Specialised-kernel paths on [B, 90, 180, 768] bf16 (the FourCastNet AFNO W-transforms, the
    16-byte-lane afno_wfft kernels; the fixed-Stockham NADD = 3 alternative is a tuning-build A/B)."""
    x, pre, g, b = _inputs(B=2, H=90, W=180, C=768, seed=2)
    xb = x.to(torch.bfloat16)
    p = pre if with_pre else None
    st = ops.ln_stats(xb.to(device), None if p is None else p.to(device), 1e-6)
    st_ref = ops.ln_stats(xb, p, 1e-6)
    torch.testing.assert_close(st.cpu(), st_ref, rtol=1e-4, atol=1e-4)
    km, scale = 46, 1 / math.sqrt(90 * 180)
    dv = lambda t: None if t is None else t.to(device)  # noqa: E731
    X = ops.r2c_ln(xb.to(device), 2, scale, km, st, g.to(device), b.to(device), dv(p), torch.bfloat16)
    _, h = _ln_ref(xb, p, g, b, 1e-6)
    Xref = torch.view_as_real(torch.fft.rfft(h, dim=2)[:, :, :km] * scale)
    assert X.dtype == torch.bfloat16
    assert rel_l2(X, Xref) < 1e-2
    Y = (0.05 * torch.randn(2, 90, km, 768, 2)).to(torch.bfloat16)
    out = ops.c2r_ln_add(Y.to(device), 2, 180, scale, xb.to(device), st, g.to(device), b.to(device), dv(p))
    full = torch.zeros(2, 90, 91, 768, dtype=torch.complex128)
    full[:, :, :km] = torch.view_as_complex(Y.double())
    xp, hh = _ln_ref(xb, p, g, b, 1e-6)
    ref = scale * torch.fft.irfft(full, n=180, dim=2, norm="forward") + xp + hh
    assert out.dtype == torch.bfloat16
    assert rel_l2(out, ref) < 1e-2
    assert not [w for w in recwarn if "no specialised LayerNorm-fused kernel" in str(w.message)]


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [1, 15, 1024])
@pytest.mark.parametrize("with_pre", [False, True])
def test_ln_stats_768_kernel_gpu(device, rows, with_pre):
    """Two-rows-per-wave statistics kernel (768 channels), including an odd row count."""
    g = torch.Generator().manual_seed(rows)
    x = (3 + 2 * torch.randn(rows, 768, generator=g)).to(torch.bfloat16)
    pre = torch.randn(768, generator=g) if with_pre else None
    st = ops.ln_stats(x.to(device), None if pre is None else pre.to(device), 1e-6).cpu()
    ref = ops.ln_stats(x, pre, 1e-6)
    torch.testing.assert_close(st, ref, rtol=2e-4, atol=2e-4)
