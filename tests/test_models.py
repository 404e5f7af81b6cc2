"""Model tier (CPU): FourCastNet AFNO MI355X-path composition == FourCastNet reference."""
import pytest
import torch

from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet, afno2d_reference, flops_per_sample
from tensorrt_dft_plugins_amd.models.afno import afno2d_amd, kept_window
from tensorrt_dft_plugins_amd.ops import spectral as S
from helpers import rel_l2


def small_cfg(**kw):
    d = dict(img_size=(48, 96), patch_size=8, in_chans=4, out_chans=4, embed_dim=64, depth=2, num_blocks=4)
    d.update(kw)
    return AFNOConfig(**d)


def test_kept_window_fourcastnet():
    assert kept_window(90, 180, 1.0) == (0, 90, 46)
    assert kept_window(90, 180, 0.5) == (23, 69, 23)


@pytest.mark.parametrize("frac", [1.0, 0.5])
def test_afno2d_amd_matches_reference_cpu(frac):
    torch.manual_seed(0)
    B, H, W, C, nb = 2, 6, 12, 32, 4
    x = torch.randn(B, H, W, C)
    bs = C // nb
    w1, w2 = 0.3 * torch.randn(2, nb, bs, bs), 0.3 * torch.randn(2, nb, bs, bs)
    b1, b2 = 0.1 * torch.randn(2, nb, bs), 0.1 * torch.randn(2, nb, bs)
    ref = afno2d_reference(x, w1, b1, w2, b2, nb, 0.01, frac)
    out = afno2d_amd(x, w1, b1, w2, b2, nb, 0.01, frac)
    assert rel_l2(out, ref) < 1e-5


def test_afno_spectral_op_cpu_semantics():
    """The fused-op CPU impl == composition of FFT_H, real-block MLP, softshrink, IFFT_H."""
    torch.manual_seed(1)
    B, H, KM, C, nb = 1, 10, 3, 16, 2
    bs = C // nb
    xw = torch.randn(B, H, KM, C, 2)
    w1, w2 = 0.3 * torch.randn(2, nb, bs, bs), 0.3 * torch.randn(2, nb, bs, bs)
    b1, b2 = 0.1 * torch.randn(2, nb, bs), 0.1 * torch.randn(2, nb, bs)
    w1t, w2t, b1p, b2p = S.pack_afno_weights(w1, b1, w2, b2)
    y = torch.ops.amd_dft.afno_spectral(xw, w1t, w2t, b1p, b2p, 0.01)
    X = torch.fft.fft(torch.view_as_complex(xw), dim=1).reshape(B, H, KM, nb, bs)
    W1c = torch.complex(w1t.float()[:, :bs, :bs].transpose(1, 2), w1t.float()[:, bs:, :bs].transpose(1, 2))
    # reference in complex form with bf16-rounded weights
    w1r = w1.to(torch.bfloat16).float()
    w2r = w2.to(torch.bfloat16).float()
    o1r = torch.relu(torch.einsum("...bi,bio->...bo", X.real, w1r[0]) - torch.einsum("...bi,bio->...bo", X.imag, w1r[1]) + b1[0])
    o1i = torch.relu(torch.einsum("...bi,bio->...bo", X.imag, w1r[0]) + torch.einsum("...bi,bio->...bo", X.real, w1r[1]) + b1[1])
    o2r = torch.einsum("...bi,bio->...bo", o1r, w2r[0]) - torch.einsum("...bi,bio->...bo", o1i, w2r[1]) + b2[0]
    o2i = torch.einsum("...bi,bio->...bo", o1i, w2r[0]) + torch.einsum("...bi,bio->...bo", o1r, w2r[1]) + b2[1]
    o = torch.nn.functional.softshrink(torch.stack([o2r, o2i], -1), 0.01)
    ref = torch.fft.ifft(torch.view_as_complex(o.contiguous()).reshape(B, H, KM, C), dim=1, norm="forward")
    assert rel_l2(torch.view_as_complex(y), ref) < 1e-5
    assert W1c.shape == (nb, bs, bs)


def test_afnonet_backends_agree_cpu():
    torch.manual_seed(2)
    cfg = small_cfg()
    m = AFNONet(cfg, backend="torch").eval()
    x = torch.randn(2, cfg.in_chans, *cfg.img_size)
    with torch.no_grad():
        ref = m(x)
        out = m.set_backend("amd")(x)
    assert out.shape == (2, cfg.out_chans, *cfg.img_size)
    assert rel_l2(out, ref) < 1e-4


def test_layer_norm_op_cpu():
    x = torch.randn(5, 64).to(torch.bfloat16)
    r = torch.randn(5, 64).to(torch.bfloat16)
    ln = torch.nn.LayerNorm(64)
    y, xs = S.layer_norm(x, ln, r)
    ref = torch.nn.functional.layer_norm((x.float() + r.float()), (64,), ln.weight, ln.bias, ln.eps)
    assert rel_l2(y.float(), ref) < 1e-2
    assert torch.allclose(xs.float(), (x.float() + r.float()).to(torch.bfloat16).float())


def test_fourcastnet_flops():
    f = flops_per_sample(AFNOConfig())
    assert 1.8e12 < f < 2.1e12  # ~2.0 TFLOP/sample


def test_afno_fused_shape_table_matches_native():
    from tensorrt_dft_plugins_amd.ops.spectral import AFNO_FUSED_SHAPES

    for H in (32, 45, 64, 90, 180):
        for bs in (48, 64, 96, 128):
            assert bool(torch.ops.amd_dft.afno_spectral_supported(H, bs)) == ((H, bs) in AFNO_FUSED_SHAPES)
    listed = list(torch.ops.amd_dft.afno_spectral_shapes())
    assert set(zip(listed[0::2], listed[1::2])) == set(AFNO_FUSED_SHAPES)
