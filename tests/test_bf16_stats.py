"""bf16 FourCastNet block without LayerNorm-statistics passes: the fc2 epilogue (linear_stats) and the
AFNO C2R epilogue (c2r_ln_add_part) emit the next LayerNorm's per-64-channel partials of the STORED
(bf16-rounded) outputs; ln_stats_merge turns them into (mean, rstd).  Each op against its plain
PyTorch form (linear / c2r_ln_add + fp64 statistics of the stored tensor)."""
import math

import pytest
import torch
import torch.nn.functional as F

from helpers import rel_l2
from tensorrt_dft_plugins_amd.ops import spectral as S

ops = torch.ops.amd_dft


def _ln_stats_ref(y, pre=None):
    v = y.double() + (0 if pre is None else pre.double())
    return torch.stack([v.mean(-1), torch.rsqrt(v.var(-1, unbiased=False) + 1e-6)], -1).float()


# ------------------------------------------------------------------ CPU semantics
def test_linear_stats_cpu_semantics():
    torch.manual_seed(21)
    x, w = torch.randn(37, 128).bfloat16(), (torch.randn(256, 128) * 0.1).bfloat16()
    r, pre = torch.randn(37, 256).bfloat16(), torch.randn(256)
    y, part = ops.linear_stats(x, w, r, pre)
    assert y.dtype == torch.bfloat16 and part.shape == (37, 4, 2)
    assert torch.equal(y, ops.linear(x, w, None, 0, r))
    st = ops.ln_stats_merge(part, 1e-6)
    assert torch.allclose(st, _ln_stats_ref(y.float(), pre), rtol=1e-5, atol=1e-6)
    yo, po = ops.linear_stats(torch.empty(5, 3072, device="meta", dtype=torch.bfloat16),
                              torch.empty(768, 3072, device="meta", dtype=torch.bfloat16),
                              torch.empty(5, 768, device="meta", dtype=torch.bfloat16))
    assert yo.shape == (5, 768) and yo.dtype == torch.bfloat16 and po.shape == (5, 12, 2)


def test_c2r_ln_add_part_cpu_semantics():
    torch.manual_seed(22)
    B, H, W, C = 1, 3, 180, 128
    x = torch.randn(B, H, W, C).bfloat16()
    g, be, pre = torch.randn(C) * 0.3 + 1, torch.randn(C) * 0.1, torch.randn(C) * 0.2
    st = ops.ln_stats(x, pre, 1e-6)
    X = torch.randn(B, H, 46, C, 2).bfloat16()
    y, part = ops.c2r_ln_add_part(X, 2, W, 0.01, x, st, g, be, pre)
    assert torch.equal(y, ops.c2r_ln_add(X, 2, W, 0.01, x, st, g, be, pre))
    assert part.shape == (B * H * W, C // 64, 2)
    st2 = ops.ln_stats_merge(part, 1e-6)
    assert torch.allclose(st2, _ln_stats_ref(y.float().reshape(-1, C)), rtol=1e-5, atol=1e-6)
    with pytest.raises(RuntimeError, match="bf16"):
        ops.c2r_ln_add_part(X.float(), 2, W, 0.01, x.float(), st, g, be, pre)
    yo, po = ops.c2r_ln_add_part(torch.empty(2, 90, 46, 768, 2, device="meta", dtype=torch.bfloat16), 2, 180, 1.0,
                                 torch.empty(2, 90, 180, 768, device="meta", dtype=torch.bfloat16),
                                 torch.empty(2 * 90 * 180, 2, device="meta"), torch.empty(768, device="meta"),
                                 torch.empty(768, device="meta"))
    assert yo.shape == (2, 90, 180, 768) and po.shape == (2 * 90 * 180, 12, 2)


# ------------------------------------------------------------------ GPU kernels
@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K,with_pre", [(777, 768, 3072, True), (300, 256, 64, False), (1, 512, 128, True)])
def test_linear_stats_gpu(device, M, N, K, with_pre):
    """fc2's bf16 statistics epilogue (staged rounded outputs + pre, one lane per token row; ragged M):
    the output is bit-identical to the plain hand GEMM's, the merged statistics match fp64 statistics
    of the stored output + pre, and ln_stats over that output."""
    torch.manual_seed(M + N + K)
    d = lambda t: None if t is None else t.to(device)  # noqa: E731
    x, w = torch.randn(M, K).bfloat16(), (torch.randn(N, K) / K ** 0.5).bfloat16()
    r = (torch.randn(M, N) * 3 + 1).bfloat16()
    pre = torch.randn(N) * 0.5 if with_pre else None
    S.fallback_reset()
    y, part = ops.linear_stats(d(x), d(w), d(r), d(pre))
    assert S.fallback_counts() == {}
    assert part.shape == (M, N // 64, 2)
    assert torch.equal(y, ops.linear(d(x), d(w), None, 0, d(r)))
    assert rel_l2(y.float().cpu(), F.linear(x.float(), w.float()) + r.float()) < 1e-2
    st = ops.ln_stats_merge(part, 1e-6).cpu()
    ref = _ln_stats_ref(y.float().cpu(), pre)
    assert torch.allclose(st, ref, rtol=2e-5, atol=2e-6), (st - ref).abs().max()
    assert torch.allclose(st, ops.ln_stats(y, d(pre), 1e-6).cpu(), rtol=2e-5, atol=2e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("with_pre", [False, True])
def test_c2r_ln_add_part_gpu(device, with_pre):
    """The bf16 AFNO C2R epilogue's LN partials (the stored bf16 values staged in the idle FFT buffer,
    one thread per position): output bit-identical to c2r_ln_add's, merged statistics vs fp64."""
    torch.manual_seed(23)
    B, H, W, C = 2, 90, 180, 768
    d = lambda t: None if t is None else t.to(device)  # noqa: E731
    x = (torch.randn(B, H, W, C) + 0.5).bfloat16()
    g, be = torch.randn(C) * 0.3 + 1, torch.randn(C) * 0.1
    pre = torch.randn(C) * 0.2 if with_pre else None
    st = ops.ln_stats(d(x), d(pre), 1e-6)
    X = torch.randn(B, H, 46, C, 2).bfloat16()
    sc = 1.0 / math.sqrt(H * W)
    S.fallback_reset()
    y, part = ops.c2r_ln_add_part(d(X), 2, W, sc, d(x), st, d(g), d(be), d(pre))
    assert S.fallback_counts() == {}
    assert torch.equal(y, ops.c2r_ln_add(d(X), 2, W, sc, d(x), st, d(g), d(be), d(pre)))
    stg = ops.ln_stats_merge(part, 1e-6).cpu()
    sref = _ln_stats_ref(y.float().cpu().reshape(-1, C))
    assert torch.allclose(stg, sref, rtol=2e-5, atol=2e-6), (stg - sref).abs().max()
    assert torch.allclose(stg, ops.ln_stats(y, None, 1e-6).cpu(), rtol=2e-5, atol=2e-6)
