"""FNO model family: SpectralConv2d / FNO block / FNO2d on the amd ops vs the torch.fft oracle
(CPU tier here; the GPU tier runs the same checks on the native kernels)."""
import pytest
import torch
import torch.nn.functional as F

from tensorrt_dft_plugins_amd.models import FNO2d, FNOBlock, FNOConfig, spectral_conv2d_reference
from tensorrt_dft_plugins_amd.ops import spectral as S
from helpers import rel_l2


def _block(width, m1, m2, seed=0):
    torch.manual_seed(seed)
    return FNOBlock(width, m1, m2, backend="torch")


def test_spectral_conv_reference_matches_dense_definition():
    """The oracle against a dense complex-DFT formulation (independent of slicing conventions)."""
    torch.manual_seed(0)
    B, C, H, W, m1, m2 = 1, 3, 8, 10, 2, 3
    x = torch.randn(B, C, H, W, dtype=torch.float64)
    wt = torch.randn(C, C, 2 * m1, m2, 2, dtype=torch.float64)
    xf = torch.fft.fft2(x)
    wc = torch.view_as_complex(wt)
    out = torch.zeros(B, C, H, W, dtype=torch.complex128)
    for kx in list(range(m1)) + list(range(H - m1, H)):
        r = kx if kx < m1 else kx - (H - m1) + m1
        for ky in range(m2):
            v = torch.einsum("bi,io->bo", xf[:, :, kx, ky], wc[:, :, r, ky])
            out[:, :, kx, ky] = v
    ref = spectral_conv2d_reference(x.float(), wt.float(), m1, m2)
    half = torch.zeros(B, C, H, W // 2 + 1, dtype=torch.complex128)
    half[..., :m2] = out[..., :m2]
    assert rel_l2(ref, torch.fft.irfft2(half, s=(H, W))) < 1e-5


@pytest.mark.parametrize("shape", [(2, 4, 16, 24, 3, 5), (1, 20, 36, 40, 6, 8)])
def test_spectral_conv_amd_cpu(shape):
    B, C, H, W, m1, m2 = shape
    torch.manual_seed(1)
    blk = _block(C, m1, m2)
    x = torch.randn(B, C, H, W)
    ref = blk.spectral(x)
    blk.spectral.backend = "amd"
    out = blk.spectral(x)
    assert rel_l2(out, ref) < 1e-5


def test_fno_mix_op_cpu():
    torch.manual_seed(2)
    xm = torch.randn(3, 5, 7, 2)
    w = torch.randn(5, 4, 7, 2)
    y = torch.ops.amd_dft.fno_mix(xm, w)
    ref = torch.einsum("bim,iom->bom", torch.view_as_complex(xm), torch.view_as_complex(w))
    assert rel_l2(torch.view_as_complex(y.contiguous()), ref) < 1e-6


def test_fno_pointwise_op_cpu():
    torch.manual_seed(3)
    x = torch.randn(2, 20, 6, 8)
    s = torch.randn(2, 20, 6, 8)
    w = torch.randn(20, 20)
    b = torch.randn(20)
    y = torch.ops.amd_dft.fno_pointwise(s, x, w, b, True)
    assert rel_l2(y, F.gelu(F.conv2d(x, w[:, :, None, None], b) + s)) < 1e-6
    y2 = torch.ops.amd_dft.fno_pointwise(None, x, w[:8], b[:8], False)
    assert y2.shape == (2, 8, 6, 8)
    assert rel_l2(y2, F.conv2d(x, w[:8, :, None, None], b[:8])) < 1e-6


def test_fno_block_amd_cpu():
    torch.manual_seed(4)
    blk = _block(20, 4, 5)
    x = torch.randn(2, 20, 24, 32)
    with torch.no_grad():
        ref = blk(x)
        blk.backend = blk.spectral.backend = "amd"
        out = blk(x)
    assert rel_l2(out, ref) < 1e-5


def test_fno2d_amd_cpu():
    torch.manual_seed(5)
    cfg = FNOConfig(img_size=(32, 48), in_chans=4, out_chans=3, width=16, modes1=5, modes2=7, n_layers=3,
                    proj_hidden=32)
    m = FNO2d(cfg, backend="torch").eval()
    x = torch.randn(2, 4, 32, 48)
    with torch.no_grad():
        ref = m(x)
        out = m.set_backend("amd")(x)
    assert out.shape == (2, 3, 32, 48)
    assert rel_l2(out, ref) < 1e-5


def test_spectral_mix_fallback_matches():
    torch.manual_seed(6)
    xm = torch.randn(2, 3, 10, 2)
    w = torch.randn(3, 3, 10, 2)
    assert rel_l2(S.fno_spectral_mix(xm, w), torch.ops.amd_dft.fno_mix(xm, w)) < 1e-6


def test_modes_too_large():
    blk = _block(4, 20, 5)
    blk.backend = blk.spectral.backend = "amd"
    with pytest.raises(ValueError):
        blk(torch.randn(1, 4, 16, 16))


@pytest.mark.gpu
def test_fno_mix_kernel_gpu(device):
    torch.manual_seed(7)
    for B, Ci, Co, M in [(1, 20, 20, 2048), (4, 20, 20, 100), (32, 20, 20, 37), (3, 7, 5, 19), (2, 32, 16, 64),
                         (12, 20, 20, 64), (8, 20, 20, 2048)]:
        xm = torch.randn(B, Ci, M, 2)
        w = torch.randn(Ci, Co, M, 2)
        ref = torch.ops.amd_dft.fno_mix(xm, w)
        out = torch.ops.amd_dft.fno_mix(xm.to(device), w.to(device))
        assert rel_l2(out, ref) < 1e-5, (B, Ci, Co, M)


@pytest.mark.gpu
def test_fno_pointwise_kernel_gpu(device):
    torch.manual_seed(8)
    for dt in (torch.float32, torch.bfloat16):
        for (B, Ci, Co, H, W) in [(2, 20, 20, 72, 144), (1, 20, 128, 9, 7), (1, 128, 20, 8, 8), (3, 4, 6, 5, 3)]:
            x = torch.randn(B, Ci, H, W).to(dt)
            s = torch.randn(B, Co, H, W).to(dt)
            w = torch.randn(Co, Ci) / Ci ** 0.5
            b = torch.randn(Co)
            ref = torch.ops.amd_dft.fno_pointwise(s.float(), x.float(), w, b, True)
            out = torch.ops.amd_dft.fno_pointwise(s.to(device), x.to(device), w.to(device), b.to(device), True)
            assert out.dtype == dt
            assert rel_l2(out.float(), ref) < (1e-5 if dt == torch.float32 else 1e-2), (dt, B, Ci, Co, H, W)


@pytest.mark.gpu
def test_fno_block_gpu_full_grid(device):
    """BASELINE config 3: FNO SpectralConv2d block, 20 ch, 720x1440, bf16 (and fp32)."""
    torch.manual_seed(9)
    blk = _block(20, 32, 32).to(device)
    x = torch.randn(1, 20, 720, 1440, device=device)
    with torch.no_grad():
        ref = blk(x)
        blk.backend = blk.spectral.backend = "amd"
        out = blk(x)
        assert rel_l2(out, ref) < 1e-4
        outb = blk(x.to(torch.bfloat16))
    assert outb.dtype == torch.bfloat16
    assert rel_l2(outb.float(), ref) < 2e-2


@pytest.mark.gpu
def test_fno2d_gpu(device):
    torch.manual_seed(10)
    cfg = FNOConfig(img_size=(90, 180), modes1=12, modes2=12, n_layers=2)
    m = FNO2d(cfg, backend="torch").to(device).eval()
    x = torch.randn(2, 20, 90, 180, device=device)
    with torch.no_grad():
        ref = m(x)
        out = m.set_backend("amd")(x)
    assert rel_l2(out, ref) < 1e-4


def test_c2c_axis_cpu():
    torch.manual_seed(11)
    x = torch.randn(2, 3, 10, 4, 2)
    full = torch.fft.fft(torch.view_as_complex(x).to(torch.complex128), dim=2)
    y = torch.ops.amd_dft.c2c_axis(x, 2, 10, 10, 0, 3, 2, False, 1.0)
    ref = torch.cat([full[:, :, :3], full[:, :, -2:]], 2)
    assert rel_l2(torch.view_as_complex(y.contiguous()), ref) < 1e-6
    z = torch.ops.amd_dft.c2c_axis(y, 2, 10, 3, 2, 10, 0, True, 0.1)
    pad = torch.zeros(2, 3, 10, 4, dtype=torch.complex128)
    pad[:, :, :3] = ref[:, :, :3]
    pad[:, :, -2:] = ref[:, :, 3:]
    assert rel_l2(torch.view_as_complex(z.contiguous()), torch.fft.ifft(pad, dim=2)) < 1e-6


def test_dftw_r2c_cpu():
    x = torch.randn(3, 64)
    y = torch.ops.amd_dft.dftw_r2c(x, 9, 0.5)
    ref = 0.5 * torch.fft.rfft(x.double())[:, :9]
    assert rel_l2(torch.view_as_complex(y.contiguous()), ref) < 1e-6


def test_fno_c2r_cpu():
    """fno_c2r: the layer tail without its pointwise branch = irfft along W of the kept modes."""
    torch.manual_seed(13)
    B, Co, H, W, m = 2, 3, 4, 16, 6
    yw = torch.randn(B, Co, H, m, 2)
    full = torch.zeros(B, Co, H, W // 2 + 1, dtype=torch.complex128)
    full[..., :m] = torch.view_as_complex(yw.double())
    ref = torch.fft.irfft(full, n=W, dim=3, norm="forward")
    y = torch.ops.amd_dft.fno_c2r(yw, W)
    assert y.dtype == torch.float32 and y.shape == (B, Co, H, W)
    assert rel_l2(y, ref) < 1e-6
    yb = torch.ops.amd_dft.fno_c2r(yw, W, torch.bfloat16)
    assert yb.dtype == torch.bfloat16 and rel_l2(yb.float(), ref) < 1e-2
    with pytest.raises(RuntimeError):
        torch.ops.amd_dft.fno_c2r(yw, 8)  # 6 modes need W >= 10
    assert torch.ops.amd_dft.fno_c2r(yw.to("meta"), W, torch.bfloat16).shape == (B, Co, H, W)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_fno_c2r_kernel_gpu(device, dt):
    """The spectral-only tail kernel (fno_c2r_pw without x / conv / activation) vs the fp64 irfft, at the
    FNO grid (720 x 1440, 32 modes, 20 channels) and a ragged one (W not a multiple of the chunk)."""
    torch.manual_seed(14)
    for B, Co, H, W, m in [(1, 20, 720, 1440, 32), (2, 5, 9, 200, 17)]:
        yw = torch.randn(B, Co, H, m, 2) / (H * W) ** 0.5
        ref = torch.ops.amd_dft.fno_c2r(yw, W)
        y = torch.ops.amd_dft.fno_c2r(yw.to(device), W, dt)
        assert y.dtype == dt and y.shape == (B, Co, H, W)
        assert rel_l2(y.float().cpu(), ref) < (2e-5 if dt == torch.float32 else 8e-3), (B, Co, H, W, m)


@pytest.mark.gpu
def test_fno_c2r_unaligned_view_gpu(device):
    """The tail reads 4 modes per 16-byte load: a spectrum view starting 8 bytes into its storage still works."""
    torch.manual_seed(16)
    B, Co, H, W, m = 1, 20, 6, 1440, 32
    flat = torch.randn(B * Co * H * m * 2 + 2, device=device)
    yw = flat[2:].view(B, Co, H, m, 2)
    assert yw.data_ptr() % 16 == 8
    ref = torch.ops.amd_dft.fno_c2r(yw.cpu(), W)
    for dt in (torch.float32, torch.bfloat16):
        y = torch.ops.amd_dft.fno_c2r(yw, W, dt)
        assert rel_l2(y.float().cpu(), ref) < (2e-5 if dt == torch.float32 else 8e-3)
    x = torch.randn(B, 4, H, W, device=device)
    wc = torch.randn(Co, 4, device=device)
    y = torch.ops.amd_dft.fno_c2r_pw(yw, x, wc, None, False)
    refp = torch.ops.amd_dft.fno_c2r_pw(yw.cpu(), x.cpu(), wc.cpu(), None, False)
    assert rel_l2(y.cpu(), refp) < 2e-5


@pytest.mark.gpu
def test_spectral_conv2d_gpu_full_grid(device):
    """BASELINE config 3's SpectralConv2d alone (rfft2 -> per-mode complex mixing -> irfft2), 20 ch,
    720 x 1440, modes 32 x 32, on the amd kernels vs the plain-PyTorch reference (fp32 and bf16)."""
    torch.manual_seed(15)
    blk = _block(20, 32, 32).to(device)
    sp = blk.spectral
    x = torch.randn(1, 20, 720, 1440, device=device)
    with torch.no_grad():
        ref = sp(x)
        sp.backend = "amd"
        out = sp(x)
        outb = sp(x.to(torch.bfloat16))
    assert out.dtype == torch.float32 and rel_l2(out, ref) < 1e-4
    assert outb.dtype == torch.bfloat16 and rel_l2(outb.float(), ref) < 2e-2


def test_fno_c2r_pw_cpu():
    torch.manual_seed(12)
    B, Ci, Co, H, W, m = 2, 5, 3, 4, 16, 6
    yw = torch.randn(B, Co, H, m, 2)
    x = torch.randn(B, Ci, H, W)
    wc = torch.randn(Co, Ci)
    b = torch.randn(Co)
    y = torch.ops.amd_dft.fno_c2r_pw(yw, x, wc, b, True)
    full = torch.zeros(B, Co, H, W // 2 + 1, dtype=torch.complex128)
    full[..., :m] = torch.view_as_complex(yw.double())
    spec = torch.fft.irfft(full, n=W, dim=3, norm="forward")
    ref = F.gelu(spec + F.conv2d(x.double(), wc.double()[:, :, None, None], b.double()))
    assert rel_l2(y, ref) < 1e-6


@pytest.mark.gpu
def test_dftw_r2c_gemm_gpu(device):
    """Pruned R2C along the innermost axis takes the MFMA DFT-GEMM path; vs torch.fft (fp64)."""
    from tensorrt_dft_plugins_amd.ops import dft as D

    torch.manual_seed(13)
    for (R, W, m) in [(14400, 1440, 32), (37, 720, 16), (5, 64, 8), (100, 1440, 64), (16, 200, 20)]:
        x = torch.randn(R, W)
        ref = torch.fft.rfft(x.double(), dim=1)[:, :m]
        for dt, tol in ((torch.float32, 1e-5), (torch.bfloat16, 2e-6)):
            xd = x.to(dt)
            refd = torch.fft.rfft(xd.double(), dim=1)[:, :m]
            if dt == torch.bfloat16:  # automatic for bf16 inputs
                out = D.rfftn_pruned(xd.to(device), [1], [(m, 0)])
            else:  # explicit op for fp32 (bf16x3 split operands)
                out = torch.ops.amd_dft.dftw_r2c(xd.to(device), m, 1.0)
            assert out.shape == (R, m, 2)
            assert rel_l2(torch.view_as_complex(out.cpu().contiguous()), refd) < tol, (R, W, m, dt)


@pytest.mark.gpu
def test_fno_c2r_pw_kernel_gpu(device):
    torch.manual_seed(14)
    for (B, Ci, Co, H, W, m, gelu) in [(1, 20, 20, 8, 1440, 32, True), (2, 7, 13, 3, 200, 20, False),
                                       (1, 32, 32, 2, 720, 64, True), (3, 4, 16, 5, 64, 5, True)]:
        yw = torch.randn(B, Co, H, m, 2) / W
        wc = torch.randn(Co, Ci) / Ci ** 0.5
        b = torch.randn(Co)
        for dt, tol in ((torch.float32, 2e-5), (torch.bfloat16, 1e-2)):
            x = torch.randn(B, Ci, H, W).to(dt)
            ref = torch.ops.amd_dft.fno_c2r_pw(yw, x.float(), wc, b, gelu)
            out = torch.ops.amd_dft.fno_c2r_pw(yw.to(device), x.to(device), wc.to(device), b.to(device), gelu)
            assert out.dtype == dt
            assert rel_l2(out.float(), ref) < tol, (B, Ci, Co, H, W, m, dt)


def _mix_c2c_reference(xm, w, n, lo, hi, scale):
    """fp64 torch composition: complex mode mixing, zero-padded unnormalised inverse FFT along dim 2."""
    B, Ci, S_, I, _ = xm.shape
    Co = w.shape[1]
    xc = torch.view_as_complex(xm.double().contiguous())
    wc = torch.view_as_complex(w.double().reshape(Ci, Co, S_, I, 2).contiguous())
    ym = torch.einsum("bisc,iosc->bosc", xc, wc)
    full = torch.zeros(B, Co, n, I, dtype=torch.complex128)
    full[:, :, :lo] = ym[:, :, :lo]
    if hi:
        full[:, :, n - hi:] = ym[:, :, lo:]
    return torch.view_as_real(torch.fft.ifft(full, dim=2, norm="forward") * scale)


@pytest.mark.parametrize("shape", [(1, 4, 5, 20, 3, 3, 6), (2, 3, 2, 16, 4, 2, 3)])
def test_fno_mix_c2c_cpu(shape):
    """Mode mixing + pruned inverse C2C in one op (CPU: fno_mix + c2c_axis) vs the fp64 composition."""
    B, Ci, Co, n, lo, hi, I = shape
    torch.manual_seed(21)
    xm = torch.randn(B, Ci, lo + hi, I, 2)
    w = torch.randn(Ci, Co, (lo + hi) * I, 2)
    out = torch.ops.amd_dft.fno_mix_c2c(xm, w, n, lo, hi, 0.25)
    assert out.shape == (B, Co, n, I, 2)
    assert rel_l2(out, _mix_c2c_reference(xm, w, n, lo, hi, 0.25)) < 1e-6


@pytest.mark.gpu
def test_fno_mix_c2c_gpu(device):
    """Fused mixing gather of the fixed 720-point column kernel (FNO config 3 shapes) and the
    unfused fallback (a length with no fixed column kernel), vs the fp64 composition."""
    torch.manual_seed(22)
    for (B, Ci, Co, n, lo, hi, I) in [(1, 20, 20, 720, 32, 32, 32), (2, 7, 13, 720, 12, 12, 9), (1, 5, 6, 50, 4, 4, 7)]:
        xm = torch.randn(B, Ci, lo + hi, I, 2)
        w = torch.randn(Ci, Co, (lo + hi) * I, 2)
        ref = _mix_c2c_reference(xm, w, n, lo, hi, 1.0 / n)
        out = torch.ops.amd_dft.fno_mix_c2c(xm.to(device), w.to(device), n, lo, hi, 1.0 / n)
        assert rel_l2(out.cpu(), ref) < 2e-6, (B, Ci, Co, n, lo, hi, I)


@pytest.mark.gpu
@pytest.mark.parametrize("path", [1, 2])
def test_fno_mix_c2c_paths_gpu(device, path):
    """Both mixing paths of fno_mix_c2c at a batched FNO shape (B = 8): the gather inside the inverse
    H transform (1) and the batched MFMA GEMM + pruned inverse C2C (2), vs the fp64 composition."""
    torch.manual_seed(23)
    B, Ci, Co, n, lo, hi, I = 8, 20, 20, 720, 32, 32, 32
    xm = torch.randn(B, Ci, lo + hi, I, 2)
    w = torch.randn(Ci, Co, (lo + hi) * I, 2)
    ref = _mix_c2c_reference(xm, w, n, lo, hi, 1.0 / n)
    out = torch.ops.amd_dft.fno_mix_c2c(xm.to(device), w.to(device), n, lo, hi, 1.0 / n, path)
    assert rel_l2(out.cpu(), ref) < 2e-6


@pytest.mark.gpu
@pytest.mark.parametrize("mix_path", [1, 2])
def test_fno_block_batched_mfma_mix_gpu(device, mix_path):
    """The FNO block at batch 8 with the mode mixing on the batched MFMA kernel (2) and in the
    gather (1) against the plain-PyTorch SpectralConv2d reference (spectral_conv2d_reference + conv
    + GELU); no ATen fallback on either path."""
    from tensorrt_dft_plugins_amd.ops import spectral as S

    torch.manual_seed(24)
    blk = _block(20, 32, 32).to(device)
    x = torch.randn(8, 20, 720, 1440, device=device)
    with torch.no_grad():
        ref = blk(x)
        blk.backend = blk.spectral.backend = "amd"
        blk.mix_path = mix_path
        S.fallback_reset()
        out = blk(x)
    assert S.fallback_counts() == {}
    assert rel_l2(out, ref) < 1e-4
