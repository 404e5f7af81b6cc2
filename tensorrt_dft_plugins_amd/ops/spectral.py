"""Fused spectral-layer ops (FourCastNet AFNO, FNO) and fused LayerNorm.

``afno_spectral_h`` runs the K5 kernel of SURVEY §2.5: FFT along H -> block-diagonal complex
MLP on MFMA (bf16 operands, fp32 accumulation) -> softshrink -> inverse FFT along H, one
launch, spectrum kept in LDS.  ``c2r_w_add`` is the W-direction C2R pass with the AFNO
filter bias (and the block residual) fused into its store.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from .._loader import load_plugins
from . import dft as D

__all__ = ["pack_afno_weights", "afno_fused_available", "afno_spectral_h", "c2r_w_add", "layer_norm",
           "afno_block_amd", "afno_block_spectral", "afno_block_mlp", "fno_spectral_mix"]


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
    """fc + GELU with the activation fused into the GEMM epilogue (hipBLASLt) when available."""
    if y2.is_cuda and fc.bias is not None and hasattr(torch, "_addmm_activation"):
        return torch._addmm_activation(fc.bias, y2, fc.weight.t(), use_gelu=True)
    return F.gelu(F.linear(y2, fc.weight, fc.bias))


def afno_block_amd(blk, x: torch.Tensor, pending: Optional[torch.Tensor] = None):
    """One FourCastNet block on the MI355X path (bf16 activations).

    Residual-stream fusion: the block returns ``(x, y)`` with the true block output being
    ``x + y`` (``y`` = fc2 output incl. bias).  The addition is fused into the next block's
    LN1 (which also writes the summed residual stream), so fc2 needs no residual GEMM input
    (hipBLASLt would copy it into the output first) and no separate bias/residual kernels.
    """
    x, yn = afno_block_spectral(blk, x, pending)
    return x, afno_block_mlp(blk, yn)


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
