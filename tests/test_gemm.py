"""Fused-epilogue bf16 GEMM (csrc/nn/gemm.hip) vs an fp32 PyTorch reference."""
import pytest
import torch
import torch.nn.functional as F

from helpers import rel_l2


def _ref(x, w, b, act, r):
    y = F.linear(x.float(), w.float(), None if b is None else b.float())
    if act == 1:
        y = F.gelu(y)
    if r is not None:
        y = y + r.float()
    return y


def test_linear_cpu_semantics():
    torch.manual_seed(0)
    x = torch.randn(5, 64)
    w = torch.randn(256, 64)
    b = torch.randn(256)
    r = torch.randn(5, 256)
    y = torch.ops.amd_dft.linear(x, w, b, 1, r)
    assert rel_l2(y, _ref(x, w, b, 1, r)) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K,act,bias,res", [
    (1000, 3072, 768, 1, True, False),   # FourCastNet fc1 shape (fewer rows)
    (777, 768, 3072, 0, True, True),     # fc2 + residual, ragged M
    (256, 256, 64, 0, False, False),
    (300, 1280, 768, 0, True, False),    # head
    (33, 512, 128, 1, True, True),
])
def test_linear_gemm_gpu(device, M, N, K, act, bias, res):
    torch.manual_seed(M + N + K)
    x = (torch.randn(M, K) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N) * 0.1 if bias else None
    r = torch.randn(M, N).to(torch.bfloat16) if res else None
    ref = _ref(x, w, b, act, r)
    y = torch.ops.amd_dft.linear(x.to(device), w.to(device), None if b is None else b.to(device), act,
                                 None if r is None else r.to(device))
    assert y.dtype == torch.bfloat16 and y.shape == (M, N)
    assert rel_l2(y.float().cpu(), ref) < 6e-3


@pytest.mark.gpu
def test_linear_gemm_asymmetric_exact(device):
    """Integer operands (exact in bf16/fp32): catches transposed / permuted fragment maps."""
    M, N, K = 256, 256, 128
    x = torch.randint(-2, 3, (M, K)).to(torch.bfloat16)
    w = torch.randint(-2, 3, (N, K)).to(torch.bfloat16)
    w[0, :] = 0
    w[0, 5] = 1  # y[:, 0] = x[:, 5]
    y = torch.ops.amd_dft.linear(x.to(device), w.to(device), None, 0, None).float().cpu()
    ref = x.float() @ w.float().t()
    assert torch.equal(y, ref)
    assert torch.equal(y[:, 0], x[:, 5].float())


def _ln_fold_operands(fc_w, fc_b, gamma, beta):
    wg = (fc_w.float() * gamma.float()[None, :]).to(torch.bfloat16)
    c1 = wg.float().sum(1)
    c2 = fc_w.float() @ beta.float() + fc_b.float()
    return wg, c1, c2


def _ln_stats(x, eps):
    xf = x.float()
    return torch.stack([xf.mean(-1), torch.rsqrt(xf.var(-1, unbiased=False) + eps)], -1)


def test_linear_ln_cpu_semantics():
    """linear_ln(x) == fc(LN(x)) with the fold operands (pinned to the torch composition)."""
    torch.manual_seed(1)
    M, K, N = 7, 64, 256
    x = torch.randn(M, K) * 2 + 0.7
    w, b = torch.randn(N, K) / 8, torch.randn(N)
    g, be = torch.randn(K) * 0.2 + 1, torch.randn(K) * 0.1
    wg, c1, c2 = _ln_fold_operands(w, b, g, be)
    y = torch.ops.amd_dft.linear_ln(x, wg, c1, c2, _ln_stats(x, 1e-6), 1)
    ref = F.gelu(F.linear(F.layer_norm(x, (K,), eps=1e-6), wg.float(), c2))  # same rounded W * gamma
    ref2 = F.gelu(F.linear(F.layer_norm(x, (K,), g, be, 1e-6), w, b))
    assert rel_l2(y, ref2) < 5e-3  # bf16-rounded W * gamma
    assert rel_l2(y, ref) < 1e-5
    with pytest.raises(RuntimeError):
        torch.ops.amd_dft.linear_ln(x, wg, c1[:-1], c2, _ln_stats(x, 1e-6), 1)


@pytest.mark.gpu
@pytest.mark.parametrize("M,act", [(1000, 1), (777, 0)])
def test_linear_ln_gpu(device, M, act):
    """LN2 folded into fc1 on the hand GEMM vs LayerNorm -> linear in fp32 (FourCastNet fc1
    shape; the residual stream carries a large mean to exercise the mean * c1 correction)."""
    torch.manual_seed(M)
    K, N = 768, 3072
    x = (torch.randn(M, K) * 1.5 + 3.0).to(torch.bfloat16)
    w, b = torch.randn(N, K) / K ** 0.5, torch.randn(N) * 0.1
    g, be = torch.randn(K) * 0.2 + 1, torch.randn(K) * 0.1
    wg, c1, c2 = _ln_fold_operands(w, b, g, be)
    st = torch.ops.amd_dft.ln_stats(x.to(device), None, 1e-6)
    y = torch.ops.amd_dft.linear_ln(x.to(device), wg.to(device), c1.to(device), c2.to(device), st, act)
    assert y.dtype == torch.bfloat16 and y.shape == (M, N)
    ref = F.linear(F.layer_norm(x.float(), (K,), g, be, 1e-6), w, b)
    if act:
        ref = F.gelu(ref)
    assert rel_l2(y.float().cpu(), ref) < 8e-3


def test_linear_gelu_tanh_cpu_semantics():
    """act = 2: GELU in the tanh form (torch's approximate="tanh"), the bf16 path's option."""
    torch.manual_seed(2)
    x, w, b = torch.randn(5, 64), torch.randn(256, 64) / 8, torch.randn(256)
    y = torch.ops.amd_dft.linear(x, w, b, 2, None)
    assert rel_l2(y, F.gelu(F.linear(x, w, b), approximate="tanh")) < 1e-6
    with pytest.raises(RuntimeError):
        torch.ops.amd_dft.linear(x, w, b, 4, None)


@pytest.mark.gpu
@pytest.mark.parametrize("ln", [False, True])
def test_linear_gelu_tanh_gpu(device, ln):
    """act = 2 on the hand GEMM (FourCastNet fc1 shape, plain and LN-folded) vs torch's tanh GELU in
    fp32, and its distance from the erf form stays below bf16 resolution."""
    torch.manual_seed(11)
    M, K, N = 1000, 768, 3072
    x = (torch.randn(M, K) * 1.5 + (3.0 if ln else 0.0)).to(torch.bfloat16)
    w, b = torch.randn(N, K) / K ** 0.5, torch.randn(N) * 0.1
    if ln:
        g, be = torch.randn(K) * 0.2 + 1, torch.randn(K) * 0.1
        wg, c1, c2 = _ln_fold_operands(w, b, g, be)
        st = torch.ops.amd_dft.ln_stats(x.to(device), None, 1e-6)
        y = torch.ops.amd_dft.linear_ln(x.to(device), wg.to(device), c1.to(device), c2.to(device), st, 2)
        pre = F.linear(F.layer_norm(x.float(), (K,), g, be, 1e-6), w, b)
    else:
        wb = w.to(torch.bfloat16)
        y = torch.ops.amd_dft.linear(x.to(device), wb.to(device), b.to(device), 2, None)
        pre = F.linear(x.float(), wb.float(), b)
    yf = y.float().cpu()
    assert rel_l2(yf, F.gelu(pre, approximate="tanh")) < 8e-3
    assert (F.gelu(pre, approximate="tanh") - F.gelu(pre)).abs().max() < 5e-4  # the form's own distance


def test_linear_gelu_erf_fit_cpu_semantics():
    """act = 3: the bf16 paths' erf GELU (x sigmoid(x q(x^2)), csrc/nn/gelu.h) is within 2.6e-5 absolute of
    the exact erf GELU over the whole line, 18x closer than the tanh form."""
    x = torch.linspace(-30, 30, 600001, dtype=torch.float64).float().reshape(-1, 1)
    w = torch.ones(64, 1)  # y[:, n] = x
    y = torch.ops.amd_dft.linear(x, w, None, 3)[:, 0].double()
    exact = torch.nn.functional.gelu(x[:, 0].double())
    assert (y - exact).abs().max() < 3e-5
    tanh = torch.nn.functional.gelu(x[:, 0].double(), approximate="tanh")
    assert (tanh - exact).abs().max() > 4e-4  # the form it replaces as the bf16 default


@pytest.mark.gpu
def test_linear_gelu_erf_fit_gpu(device):
    """act = 3 on the hand GEMM (FourCastNet fc1 shape, bf16) against the exact erf GELU of the same
    pre-activation: the epilogue's form is below bf16 resolution."""
    torch.manual_seed(3)
    M, K, N = 4096, 768, 3072
    x = torch.randn(M, K, device=device).to(torch.bfloat16)
    w = (0.03 * torch.randn(N, K, device=device)).to(torch.bfloat16)
    b = 0.1 * torch.randn(N, device=device)
    y = torch.ops.amd_dft.linear(x, w, b, 3).float()
    pre = torch.nn.functional.linear(x.float(), w.float(), b)
    ref = torch.nn.functional.gelu(pre)
    assert rel_l2(y, ref) < 4e-3  # bf16 output rounding
    yt = torch.ops.amd_dft.linear(x, w, b, 2).float()
    assert rel_l2(y, ref) <= rel_l2(yt, ref)
