"""Hand GEMM with a ragged last feature panel (N % 256 != 0, N % 64 == 0) and the shapes it opens to
the hand kernels: FourCastNet at embed 384 (fc2 N = 384, AFNO block size 48) and FNO width 64,
run under ``strict_mode`` (any ATen / hipBLASLt fallback raises).

Every kernel result is compared against a plain PyTorch fp32 reference of the same op."""
import pytest
import torch
import torch.nn.functional as F

from helpers import rel_l2

pytestmark = pytest.mark.gpu


def _ref(x, w, b, act, r):
    y = F.linear(x.float(), w.float(), None if b is None else b.float())
    if act == 1:
        y = F.gelu(y)
    if r is not None:
        y = y + r.float()
    return y


@pytest.mark.parametrize("M,N,K,act,bias,res", [
    (777, 384, 1536, 0, True, True),   # FourCastNet embed-384 fc2 + residual, ragged M
    (300, 320, 128, 1, True, False),   # 256 + 64
    (513, 448, 384, 0, False, True),   # 256 + 192
    (64, 64, 64, 1, True, False),      # one half of one panel
])
def test_linear_ragged_n_bf16(device, M, N, K, act, bias, res):
    from tensorrt_dft_plugins_amd.utils import strict_mode

    torch.manual_seed(M + N + K)
    x = (torch.randn(M, K) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N) * 0.1 if bias else None
    r = torch.randn(M, N).to(torch.bfloat16) if res else None
    prev = strict_mode(True)
    try:
        y = torch.ops.amd_dft.linear(x.to(device), w.to(device), None if b is None else b.to(device), act,
                                     None if r is None else r.to(device))
    finally:
        strict_mode(prev)
    assert y.shape == (M, N)
    assert rel_l2(y.float().cpu(), _ref(x, w, b, act, r)) < 6e-3


@pytest.mark.parametrize("M,N,K,act,split_out,res", [
    (777, 384, 1536, 0, False, True),
    (500, 320, 384, 1, True, False),
    (129, 448, 128, 1, False, False),
])
def test_linear3_ragged_n(device, M, N, K, act, split_out, res):
    from tensorrt_dft_plugins_amd.ops.spectral import split_bf16, unsplit_bf16
    from tensorrt_dft_plugins_amd.utils import strict_mode

    torch.manual_seed(M * 3 + N)
    x = torch.randn(M, K, device=device)
    w = torch.randn(N, K, device=device) / K ** 0.5
    b = torch.randn(N, device=device) * 0.1
    r = torch.randn(M, N, device=device) if res else None
    prev = strict_mode(True)
    try:
        y = torch.ops.amd_dft.linear3(split_bf16(x), split_bf16(w), b, act, r, split_out)
    finally:
        strict_mode(prev)
    if split_out:
        y = unsplit_bf16(y)
    ref = _ref(x.double(), w.double(), b.double(), act, None if r is None else r.double())
    assert rel_l2(y.double().cpu(), ref.cpu()) < 2e-5


def test_linear3_stats_ragged_n(device):
    """fc2 of an embed-384 fp32 block: residual + next-LayerNorm partials over 6 chunks of 64."""
    from tensorrt_dft_plugins_amd.ops.spectral import split_bf16

    torch.manual_seed(5)
    M, K, N = 700, 1536, 384
    h = torch.randn(M, K, device=device)
    w = torch.randn(N, K, device=device) / K ** 0.5
    res = torch.randn(M, N, device=device)
    pre = torch.randn(N, device=device) * 0.1
    y, part = torch.ops.amd_dft.linear3_stats(split_bf16(h), split_bf16(w), res, pre)
    ref = (h.double() @ w.double().t() + res.double())
    assert rel_l2(y.double(), ref) < 2e-5
    chunks = (ref + pre.double()).reshape(M, N // 64, 64)
    assert rel_l2(part[..., 0].double(), chunks.mean(-1)) < 1e-5
    assert rel_l2(part[..., 1].double(), ((chunks - chunks.mean(-1, keepdim=True)) ** 2).sum(-1)) < 1e-4


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_unpatch_head_ragged(device, dtype):
    """Head GEMM + un-patchify with C = 6 output channels (N = 384): ragged GEMM + remap kernel."""
    from tensorrt_dft_plugins_amd.ops.spectral import split_bf16
    from tensorrt_dft_plugins_amd.utils import strict_mode

    torch.manual_seed(6)
    B, h, w, K, C, p = 2, 6, 10, 128, 6, 8
    t = torch.randn(B * h * w, K, device=device)
    W = torch.randn(C * p * p, K, device=device) / K ** 0.5
    bias = torch.randn(C * p * p, device=device) * 0.1
    ref = (t.double() @ W.double().t() + bias.double()).reshape(B, h, w, C, p, p).permute(0, 3, 1, 4, 2, 5)
    ref = ref.reshape(B, C, h * p, w * p)
    prev = strict_mode(True)
    try:
        if dtype == torch.float32:
            y = torch.ops.amd_dft.linear_unpatch3(split_bf16(t), split_bf16(W), bias, C, h, w, p)
            tol = 2e-5
        else:
            y = torch.ops.amd_dft.linear_unpatch(t.to(dtype), W.to(dtype), bias, C, h, w, p)
            tol = 8e-3
    finally:
        strict_mode(prev)
    assert y.shape == (B, C, h * p, w * p)
    assert rel_l2(y.double().cpu(), ref.cpu()) < tol


def test_afno_spectral_block48(device):
    """The fused H-filter at block size 48 (embed 384 / 8 blocks) vs the torch AFNO2D oracle."""
    from tensorrt_dft_plugins_amd.models.afno import AFNOConfig, afno2d_amd, afno2d_reference

    torch.manual_seed(7)
    cfg = AFNOConfig(embed_dim=384)
    C, nb = 384, 8
    x = torch.randn(2, 90, 180, C, device=device)
    w1, b1 = 0.02 * torch.randn(2, nb, 48, 48, device=device), 0.02 * torch.randn(2, nb, 48, device=device)
    w2, b2 = 0.02 * torch.randn(2, nb, 48, 48, device=device), 0.02 * torch.randn(2, nb, 48, device=device)
    ref = afno2d_reference(x, w1, b1, w2, b2, nb, 0.01, 1.0)
    for dt, tol in ((torch.float32, 2e-5), (torch.bfloat16, 3e-2)):
        y = afno2d_amd(x.to(dt), w1, b1, w2, b2, nb, 0.01, 1.0)
        assert rel_l2(y.double().cpu(), ref.double().cpu()) < tol, dt


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fourcastnet_embed384_strict(device, dtype):
    """FourCastNet at embed 384 (8 blocks of 48): every op on a hand kernel (strict mode)."""
    from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet
    from tensorrt_dft_plugins_amd.utils import strict_mode

    torch.manual_seed(8)
    cfg = AFNOConfig(embed_dim=384, depth=2)
    m = AFNONet(cfg, backend="torch").to(device).eval()
    x = torch.randn(1, cfg.in_chans, *cfg.img_size, device=device)
    with torch.no_grad():
        ref = m(x)
        m.set_backend("amd").to(dtype)
        prev = strict_mode(True)
        try:
            y = m(x.to(dtype))
        finally:
            strict_mode(prev)
    err = rel_l2(y.double().cpu(), ref.double().cpu())
    print(f"FourCastNet embed 384 {dtype}: rel-L2 vs torch fp32 {err:.3e}")
    assert err < (1e-4 if dtype == torch.float32 else 5e-2)


def test_fno2d_width64_strict(device):
    """FNO2d at width 64: hand kernels only (c2r + pointwise where the fused tail does not fit)."""
    from tensorrt_dft_plugins_amd.models import FNO2d, FNOConfig
    from tensorrt_dft_plugins_amd.utils import strict_mode

    torch.manual_seed(9)
    cfg = FNOConfig(img_size=(180, 360), width=64, modes1=16, modes2=16, n_layers=2, proj_hidden=128)
    m = FNO2d(cfg, backend="torch").to(device).eval()
    x = torch.randn(1, cfg.in_chans, *cfg.img_size, device=device)
    with torch.no_grad():
        ref = m(x)
        m.set_backend("amd")
        prev = strict_mode(True)
        try:
            y = m(x)
        finally:
            strict_mode(prev)
    assert rel_l2(y.double().cpu(), ref.double().cpu()) < 1e-4


@pytest.mark.parametrize("dtype", ["raw32", torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N", [64, 384, 768])
def test_patch_embed_ragged(device, dtype, N):
    """Patch-embedding GEMM (the image gathered in the operand DMA) with a ragged feature panel,
    + bias + position embedding; deterministic across calls and under hipGraph replay."""
    from tensorrt_dft_plugins_amd.ops.spectral import split_bf16

    torch.manual_seed(N)
    B, C, h, w, p = 2, 4, 6, 12, 8
    x = torch.randn(B, C, h * p, w * p, device=device)
    W = torch.randn(N, C * p * p, device=device) / (C * p * p) ** 0.5
    bias = torch.randn(N, device=device) * 0.1
    pos = torch.randn(h * w, N, device=device) * 0.1
    patches = x.double().reshape(B, C, h, p, w, p).permute(0, 2, 4, 1, 3, 5).reshape(B * h * w, C * p * p)
    ref = (patches @ W.double().t() + bias.double()).reshape(B, h * w, N) + pos.double()

    def run():
        if dtype == "raw32":  # the raw fp32 image (the op splits it)
            return torch.ops.amd_dft.patch_linear3(x, split_bf16(W), bias, pos, p)
        if dtype == torch.float32:
            return torch.ops.amd_dft.patch_linear3(split_bf16(x, rows=False), split_bf16(W), bias, pos, p)
        return torch.ops.amd_dft.patch_linear(x.to(dtype), W.to(dtype), bias, pos, p)

    y = run()
    assert rel_l2(y.double().reshape(B, h * w, N).cpu(), ref.cpu()) < (8e-3 if dtype == torch.bfloat16 else 2e-5)
    if dtype == "raw32":  # bit-identical to the split-planes form (same products, same order)
        assert torch.equal(y, torch.ops.amd_dft.patch_linear3(split_bf16(x, rows=False), split_bf16(W), bias, pos, p))
    assert torch.equal(run(), y)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        yg = run()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(yg, y)
