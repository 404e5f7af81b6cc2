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
