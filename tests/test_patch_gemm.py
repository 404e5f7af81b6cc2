"""Patch-embedding GEMM (patchify gather + bias + position embedding) and head GEMM
(un-patchify scatter): CPU semantics vs the FourCastNet conv / linear + permute formulation,
and the MFMA kernels (csrc/nn/gemm.hip MODE 1 / 2) vs an fp32 PyTorch reference."""
import pytest
import torch
import torch.nn.functional as F

ops = torch.ops.amd_dft


def rel_l2(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm()).item()


def _embed_ref(x, w4, bias, pos):
    """FourCastNet: Conv2d(kernel = stride = p) -> flatten -> + pos_embed."""
    y = F.conv2d(x.float(), w4.float(), bias.float(), stride=w4.shape[-1])
    t = y.flatten(2).transpose(1, 2)  # [B, h*w, N]
    return (t + pos.float().reshape(1, -1, w4.shape[0])).reshape(-1, w4.shape[0])


def _head_ref(t, w, bias, C, h, w_, p):
    """Linear -> [B, h, w, C, p, p] -> image [B, C, h*p, w*p] (feature order (c, py, px))."""
    y = F.linear(t.float(), w.float(), None if bias is None else bias.float())
    B = y.shape[0] // (h * w_)
    return y.reshape(B, h, w_, C, p, p).permute(0, 3, 1, 4, 2, 5).reshape(B, C, h * p, w_ * p)


def test_patch_linear_cpu():
    torch.manual_seed(0)
    B, C, h, w, p, N = 2, 3, 4, 5, 8, 16
    x = torch.randn(B, C, h * p, w * p)
    w4 = torch.randn(N, C, p, p) * 0.1
    bias, pos = torch.randn(N), torch.randn(h * w, N)
    y = ops.patch_linear(x, w4.reshape(N, -1), bias, pos, p)
    assert y.shape == (B * h * w, N)
    assert rel_l2(y, _embed_ref(x, w4, bias, pos)) < 1e-5


def test_linear_unpatch_cpu():
    torch.manual_seed(1)
    B, C, h, w, p, K = 2, 3, 4, 5, 8, 16
    t = torch.randn(B * h * w, K)
    wt = torch.randn(C * p * p, K) * 0.1
    bias = torch.randn(C * p * p)
    y = ops.linear_unpatch(t, wt, bias, C, h, w, p)
    assert y.shape == (B, C, h * p, w * p)
    assert rel_l2(y, _head_ref(t, wt, bias, C, h, w, p)) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("B,h,w", [(1, 90, 180), (2, 8, 40)])
def test_patch_linear_kernel_gpu(device, B, h, w):
    """MODE 1: patch gather from the image in the operand DMA + bias + broadcast pos-embed."""
    torch.manual_seed(2)
    C, p, N = 20, 8, 768
    x = torch.randn(B, C, h * p, w * p).to(torch.bfloat16)
    w4 = (torch.randn(N, C, p, p) * 0.05).to(torch.bfloat16)
    bias = torch.randn(N) * 0.1
    pos = (torch.randn(h * w, N) * 0.1).to(torch.bfloat16)
    y = ops.patch_linear(x.to(device), w4.reshape(N, -1).to(device), bias.to(device), pos.to(device), p)
    assert y.dtype == torch.bfloat16 and y.shape == (B * h * w, N)
    assert rel_l2(y, _embed_ref(x, w4, bias, pos)) < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("B,h,w", [(1, 90, 180), (2, 8, 40)])
@pytest.mark.parametrize("with_bias", [False, True])
def test_linear_unpatch_kernel_gpu(device, B, h, w, with_bias):
    """MODE 2: head GEMM with the un-patchify in its output scatter."""
    torch.manual_seed(3)
    C, p, K = 20, 8, 768
    t = torch.randn(B * h * w, K).to(torch.bfloat16)
    wt = (torch.randn(C * p * p, K) * 0.05).to(torch.bfloat16)
    bias = torch.randn(C * p * p) * 0.1 if with_bias else None
    y = ops.linear_unpatch(t.to(device), wt.to(device), None if bias is None else bias.to(device), C, h, w, p)
    assert y.dtype == torch.bfloat16 and y.shape == (B, C, h * p, w * p)
    assert rel_l2(y, _head_ref(t, wt, bias, C, h, w, p)) < 1e-2


def test_patch_linear3_raw_image_cpu_semantics():
    """patch_linear3 on the raw fp32 image equals the split-planes form (CPU reference ops)."""
    import torch

    from tensorrt_dft_plugins_amd.ops.spectral import split_bf16

    torch.manual_seed(3)
    x = torch.randn(2, 3, 16, 24)
    W = torch.randn(64, 3 * 64) * 0.1
    b, pos = torch.randn(64), torch.randn(2 * 3, 64)
    y_raw = torch.ops.amd_dft.patch_linear3(x, split_bf16(W), b, pos, 8)
    y_split = torch.ops.amd_dft.patch_linear3(split_bf16(x, rows=False), split_bf16(W), b, pos, 8)
    assert torch.allclose(y_raw, y_split, atol=1e-6)
    assert y_raw.shape == (2 * 2 * 3, 64)
