"""Fused spectral-layer ops (FourCastNet AFNO, FNO) and fused LayerNorm.

``afno_spectral_h`` runs the K5 kernel of SURVEY §2.5: FFT along H -> block-diagonal complex
MLP on MFMA (bf16 operands, fp32 accumulation) -> softshrink -> inverse FFT along H, one
launch, spectrum kept in LDS.  ``c2r_w_add`` is the W-direction C2R pass with the AFNO
filter bias (and the block residual) fused into its store.
"""
from __future__ import annotations

import math
import os
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from .._loader import load_plugins
from . import dft as D

__all__ = ["pack_afno_weights", "afno_fused_available", "afno_spectral_h", "c2r_w_add", "layer_norm",
           "afno_block_amd", "afno_block_fused", "set_mlp_backend", "mlp_on_hand_gemm", "afno_block_spectral", "afno_block_mlp", "fno_spectral_mix"]


def _ops():
    load_plugins()
    return torch.ops.amd_dft


_pack_cache: dict = {}


def _real_block(w: torch.Tensor) -> torch.Tensor:
    """[2, NB, bs, bs] complex-as-pair weight -> [NB, 2bs(k), 2bs(n)] real form [[W0, W1], [-W1, W0]]."""
    top = torch.cat([w[0], w[1]], dim=2)
    bot = torch.cat([-w[1], w[0]], dim=2)
    return torch.cat([top, bot], dim=1)


def pack_afno_weights(w1, b1, w2, b2) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """Pack AFNO2D parameters for the fused kernel: transposed real-block bf16 weights ([n][k])
    and concatenated fp32 biases.  Cached per parameter tensor version (graph-capture safe once
    warmed up)."""
    key = tuple((id(t), t.data_ptr(), t._version, str(t.device), t.dtype) for t in (w1, b1, w2, b2))
    hit = _pack_cache.get(key)
    if hit is not None:
        return hit
    with torch.no_grad():
        w1t = _real_block(w1.float()).transpose(1, 2).contiguous().to(torch.bfloat16)
        w2t = _real_block(w2.float()).transpose(1, 2).contiguous().to(torch.bfloat16)
        b1p = torch.cat([b1[0], b1[1]], dim=1).float().contiguous()
        b2p = torch.cat([b2[0], b2[1]], dim=1).float().contiguous()
    packed = (w1t, w2t, b1p, b2p)
    if len(_pack_cache) > 256:
        _pack_cache.clear()
    _pack_cache[key] = packed
    return packed


def afno_fused_available(x: torch.Tensor, num_blocks: int) -> bool:
    if not x.is_cuda:
        return False
    B, H, W, C = x.shape
    return bool(_ops().afno_spectral_supported(H, C // num_blocks))


def afno_spectral_h(xw: torch.Tensor, w1, b1, w2, b2, num_blocks: int, lam: float) -> torch.Tensor:
    w1t, w2t, b1p, b2p = pack_afno_weights(w1, b1, w2, b2)
    return _ops().afno_spectral(xw, w1t, w2t, b1p, b2p, float(lam))


def c2r_w_add(yw: torch.Tensor, x: torch.Tensor, W: int, scale: float,
              residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = scale * irfft_W(yw) + x (+ residual), with yw = [B, H, km, C, 2] (km stored modes)."""
    km = yw.shape[2]
    return _ops().c2r_add(yw, [2], [W], scale, [km, 0], x.contiguous(),
                          None if residual is None else residual.contiguous(), x.dtype)


def layer_norm(x: torch.Tensor, ln: torch.nn.LayerNorm, residual: Optional[torch.Tensor] = None):
    """Fused (x + residual) -> LayerNorm.  Returns (normed, x + residual)."""
    return _ops().layer_norm(x, ln.weight, ln.bias, ln.eps, residual)


def _gelu_linear(y2: torch.Tensor, fc: torch.nn.Linear) -> torch.Tensor:
    """fc + GELU with the activation fused into the GEMM epilogue (hipBLASLt) when available.

    hipBLASLt's GELU epilogue is the tanh approximation (measured, bench/probe_gelu.py: fp32
    max |fused - gelu_tanh| = 4.8e-7, |fused - gelu_erf| = 4.7e-4, i.e. below one bf16 ulp of
    the bf16 hidden activations for |h| > 0.06).  FourCastNet's nn.GELU is the erf form; the
    erf-exact path is the hand MFMA GEMM (``MI_DFT_MLP=hand``, erf via A&S 7.1.26, |err| < 2e-7).
    """
    if y2.is_cuda and fc.bias is not None and hasattr(torch, "_addmm_activation"):
        return torch._addmm_activation(fc.bias, y2, fc.weight.t(), use_gelu=True)
    return F.gelu(F.linear(y2, fc.weight, fc.bias))


def afno_block_amd(blk, x: torch.Tensor, pending: Optional[torch.Tensor] = None):
    """One FourCastNet block on the MI355X path (bf16 activations).

    Residual-stream fusion: the block returns ``(x, p)`` with the true block output being
    ``x + p``.  ``p`` is either a per-channel vector (the fc2 bias; LayerNorm-fused path, see
    :func:`afno_block_fused`) or a full tensor (the fc2 output; generic path, where the addition
    is fused into the next block's LN1).
    """
    if pending is not None and pending.dim() == 1 and not _ln_fused_ok(blk, x):
        x, pending = x + pending, None
    if (pending is None or pending.dim() == 1) and _ln_fused_ok(blk, x):
        return afno_block_fused(blk, x, pending)
    x, yn = afno_block_spectral(blk, x, pending)
    return x, afno_block_mlp(blk, yn)


def _f32(t: torch.Tensor) -> torch.Tensor:
    """fp32 contiguous copy of a small parameter, cached per tensor version (capture safe)."""
    key = ("f32", id(t), t.data_ptr(), t._version, str(t.device), t.dtype)
    hit = _pack_cache.get(key)
    if hit is None:
        with torch.no_grad():
            hit = t.detach().float().contiguous()
        if len(_pack_cache) > 256:
            _pack_cache.clear()
        _pack_cache[key] = hit
    return hit


def _ln_fused_ok(blk, x: torch.Tensor) -> bool:
    from ..models.afno import kept_window

    f = blk.filter
    c = f.cfg
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[-1] % 8 == 0):
        return False
    B, H, W, C = x.shape
    r0, r1, _ = kept_window(H, W, c.hard_thresholding_fraction)
    return r0 == 0 and r1 == H and afno_fused_available(x, c.num_blocks)


def afno_block_fused(blk, xs: torch.Tensor, pre: Optional[torch.Tensor] = None):
    """FourCastNet block with LN1 fused into the AFNO W-transforms and fc2 accumulated in place.

    The residual stream is carried as ``(xs, pre)`` with true x = xs + pre (pre = the previous
    block's fc2 bias, per channel, or None):

      stats = (mean, rstd) of x                  ln_stats: reads xs once, writes 8 B/token
      X_w   = R2C_W(LN1(x))                      LN applied on load (no normalised copy in HBM)
      Y_w   = FFT_H -> block MLP -> IFFT_H       afno_spectral (MFMA)
      x1    = C2R_W(Y_w) + LN1(x) + x            both skips from one read of xs
      yn    = LN2(x1); h = GELU(fc1(yn))         hipBLASLt, GELU epilogue
      x1   += h @ W2^T                           hipBLASLt beta = 1, in place (no bias pass)

    Returns (x1, fc2.bias): the bias is folded into the next block's statistics and loads
    (or the head GEMM's bias).  Saves the LN1 kernel's normalised write + residual write and
    one full-tensor read in the C2R versus :func:`afno_block_spectral`.
    """
    from ..models.afno import kept_window

    f = blk.filter
    c = f.cfg
    n1 = blk.norm1
    B, H, W, C = xs.shape
    _, _, km = kept_window(H, W, c.hard_thresholding_fraction)
    scale = 1.0 / math.sqrt(H * W)
    ops = _ops()
    pre32 = None if pre is None else _f32(pre)
    g1, be1 = _f32(n1.weight), _f32(n1.bias)
    stats = ops.ln_stats(xs, pre32, n1.eps)
    xw = ops.r2c_ln(xs, 2, scale, km, stats, g1, be1, pre32, torch.bfloat16)
    yw = afno_spectral_h(xw, f.w1, f.b1, f.w2, f.b2, c.num_blocks, c.sparsity_threshold)
    x1 = ops.c2r_ln_add(yw, 2, W, scale, xs, stats, g1, be1, pre32)
    yn, _ = layer_norm(x1, blk.norm2)
    m = blk.mlp
    if mlp_on_hand_gemm():
        # hand MFMA GEMM (csrc/nn/gemm.hip): one workgroup per output tile, no cross-workgroup
        # dependencies -- unaffected by long-lived kernels of other streams/processes (RCCL
        # collective blocks), which stall hipBLASLt's persistent stream-K grid
        hid = ops.linear(yn.reshape(-1, C), m.fc1.weight, m.fc1.bias, 1, None)
        x1 = ops.linear(hid, m.fc2.weight, None, 0, x1.reshape(-1, C)).reshape(B, H, W, C)
        return x1, m.fc2.bias
    hid = _gelu_linear(yn.reshape(-1, C), m.fc1)
    if torch.jit.is_tracing():
        x1 = torch.addmm(x1.reshape(-1, C), hid, m.fc2.weight.t()).reshape(B, H, W, C)
    else:
        x1.view(-1, C).addmm_(hid, m.fc2.weight.t())
    return x1, m.fc2.bias


_MLP_HAND: Optional[bool] = None


def set_mlp_backend(hand: Optional[bool]) -> None:
    """Force the FourCastNet MLP GEMMs onto the hand MFMA kernel (True) or hipBLASLt (False);
    None = environment / default (MI_DFT_MLP=hand|blas, default blas)."""
    global _MLP_HAND
    _MLP_HAND = hand


def mlp_on_hand_gemm() -> bool:
    if _MLP_HAND is not None:
        return _MLP_HAND
    return os.environ.get("MI_DFT_MLP", "blas") == "hand"


def afno_block_spectral(blk, x: torch.Tensor, pending: Optional[torch.Tensor] = None):
    """Bandwidth/VALU-bound half of a block: LN1(+pending residual) -> AFNO filter (+ both skips,
    fused into the C2R store) -> LN2.  Returns (residual stream x, LN2 output)."""
    from ..models.afno import afno2d_amd

    f = blk.filter
    c = f.cfg
    h, x = _ops().layer_norm(x, blk.norm1.weight, blk.norm1.bias, blk.norm1.eps, pending)
    # filter(LN1(x)) + LN1(x) [AFNO bias] + x [double skip], fused into the C2R store
    x = afno2d_amd(h, f.w1, f.b1, f.w2, f.b2, c.num_blocks, c.sparsity_threshold, c.hard_thresholding_fraction,
                   residual=x)
    yn, _ = layer_norm(x, blk.norm2)
    return x, yn


def afno_block_mlp(blk, yn: torch.Tensor) -> torch.Tensor:
    """MFMA-bound half of a block: fc1 (+bias, GELU epilogue) and fc2 (+bias) on hipBLASLt."""
    m = blk.mlp
    B, H, W, C = yn.shape
    hid = _gelu_linear(yn.reshape(-1, C), m.fc1)
    y = F.linear(hid, m.fc2.weight, m.fc2.bias)
    return y.reshape(B, H, W, C)


def fno_spectral_mix(xm: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """FNO mode mixing out[b,o,m] = sum_i x[b,i,m] w[i,o,m] on complex-as-pair tensors
    xm [B, Cin, M, 2], w [Cin, Cout, M, 2] -> [B, Cout, M, 2] (fp32).  Native op on every device
    (CPU: ATen einsum; GPU: csrc/spectral/fno_mix.hip), so it also exports as one ONNX node."""
    return _ops().fno_mix(xm.contiguous(), w.contiguous())
