"""Fused spectral-layer ops (FourCastNet AFNO, FNO) and fused LayerNorm.

``afno_spectral_h`` runs the K5 kernel of SURVEY §2.5: FFT along H -> block-diagonal complex
MLP on MFMA -> softshrink -> inverse FFT along H, one launch, spectrum kept in LDS.
``c2r_w_add`` is the W-direction C2R pass with the AFNO filter bias (and the block residual)
fused into its store.

Two precisions of the FourCastNet block run on the hand kernels:

* bf16 (``afno_block_fused``): bf16 activations, bf16 MFMA operands, fp32 accumulation.
* fp32 (``afno_block_fused_f32``, the reference's precision -- its plugins accept only
  ``kFLOAT``, /root/reference/src/dft_plugins/dft_plugins.cpp:101-102): fp32 residual stream,
  fp32 spectra and FFTs, and every GEMM as a 3-product bf16 split ("bf16x3": a = hi + lo,
  A.B = Ah.Bh + Al.Bh + Ah.Bl, fp32 accumulation; ~5e-6 relative error per GEMM against fp32
  FMA's ~3e-7 and TF32's ~1e-3) -- 3x the bf16 MFMA work, where the exact-f32 MFMA would be 16x.

Packed / split weights are cached ON THE OWNING MODULE, keyed by the parameters' storage
pointers and versions: their lifetime follows the module (a captured hipGraph that reads them
stays valid while the module lives), and a new model can never hit another model's entry.
"""
from __future__ import annotations

import math
from typing import Callable, NamedTuple, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from .._loader import load_plugins
from . import dft as D

__all__ = ["pack_afno_weights", "afno_fused_available", "afno_spectral_h", "c2r_w_add", "layer_norm",
           "afno_block_amd", "afno_block_fused", "afno_block_fused_f32",
           "afno_block_spectral", "afno_block_mlp", "fno_spectral_mix", "split_bf16", "module_cached",
           "fallback_counts", "fallback_reset", "note_fallback", "unsplit_bf16", "LnCarry", "pending_bias", "SplitRows"]


def _ops():
    load_plugins()
    return torch.ops.amd_dft


def module_cached(owner, name: str, params: Sequence[torch.Tensor], build: Callable[[], object]):
    """``build()`` cached on ``owner`` (an nn.Module) under ``name``, rebuilt when any of ``params``
    changes storage, version, dtype or device.  Superseded values stay referenced by the module
    (at most 4 per name) so graphs captured against them never read freed memory."""
    key = tuple((p.data_ptr(), p._version, p.dtype, str(p.device)) for p in params)
    cache = owner.__dict__.setdefault("_amd_packed", {})
    hit = cache.get(name)
    if hit is not None and hit[0] == key:
        return hit[1]
    with torch.no_grad():
        val = build()
    if hit is not None:
        retired = owner.__dict__.setdefault("_amd_retired", {}).setdefault(name, [])
        retired.append(hit[1])
        del retired[:-4]
    cache[name] = (key, val)
    return val


def fallback_counts() -> dict:
    """{op: calls that ran without the op's hand kernel} since the last ``fallback_reset()``."""
    names, counts = _ops().fallback_counts()
    return dict(zip(names, counts))


def fallback_reset() -> None:
    _ops().fallback_reset()


def note_fallback(op: str, why: str, x: torch.Tensor) -> None:
    """Count a GPU call of ``op`` that left the hand kernels (Python-level generic paths), in the
    same registry as the C++ ops: ``fallback_counts()`` lists it and ``MI_DFT_STRICT=1`` raises.
    CPU tensors (the reference / plumbing path) and tracing (ONNX export) are not counted."""
    if x.is_cuda and not torch.jit.is_tracing():
        _ops().fallback_note(op, why)


def split_bf16(t: torch.Tensor, rows: bool = True) -> torch.Tensor:
    """fp32 -> bf16 pair (hi = bf16(t), lo = bf16(t - hi)): rows [..., 2K] k32-interleaved (every
    32 columns stored as [hi(32) | lo(32)], the bf16x3 GEMM operand layout), or planes [2, ...]
    (``rows=False``)."""
    return _ops().split_bf16(t.float().contiguous(), rows)


def unsplit_bf16(ts: torch.Tensor) -> torch.Tensor:
    """Inverse of ``split_bf16(rows=True)``: [..., 2K] k32-interleaved pairs -> fp32 [..., K]."""
    k2 = ts.shape[-1]
    return ts.float().reshape(*ts.shape[:-1], k2 // 64, 2, 32).sum(-2).reshape(*ts.shape[:-1], k2 // 2)


def _real_block(w: torch.Tensor) -> torch.Tensor:
    """[2, NB, bs, bs] complex-as-pair weight -> [NB, 2bs(k), 2bs(n)] real form [[W0, W1], [-W1, W0]]."""
    top = torch.cat([w[0], w[1]], dim=2)
    bot = torch.cat([-w[1], w[0]], dim=2)
    return torch.cat([top, bot], dim=1)


def pack_afno_weights(w1, b1, w2, b2, split: bool = False) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor,
                                                                     torch.Tensor]:
    """AFNO2D parameters in the fused kernel's layout: transposed real-block weights ([n][k]) as
    bf16 -- or, ``split=True`` (fp32 path), as bf16 pairs [NB, n, hi k | lo k] -- and concatenated
    fp32 biases.  Pure function; callers cache the result (``module_cached``)."""
    with torch.no_grad():
        w1t = _real_block(w1.float()).transpose(1, 2).contiguous()
        w2t = _real_block(w2.float()).transpose(1, 2).contiguous()
        if split:
            w1t, w2t = split_bf16(w1t), split_bf16(w2t)
        else:
            w1t, w2t = w1t.to(torch.bfloat16), w2t.to(torch.bfloat16)
        b1p = torch.cat([b1[0], b1[1]], dim=1).float().contiguous()
        b2p = torch.cat([b2[0], b2[1]], dim=1).float().contiguous()
    return w1t, w2t, b1p, b2p


# (H, block size) instances of the fused AFNO kernel; mirrors afno_spectral_supported() in
# csrc/spectral/afno_spectral.hip (checked equal in tests/test_models.py).  Kept in Python so
# the check stays a constant under ONNX/TorchScript tracing (an op returning bool cannot be traced).
AFNO_FUSED_SHAPES = frozenset({(H, bs) for H in (45, 64, 90) for bs in (48, 64, 96, 128)})


def afno_fused_available(x: torch.Tensor, num_blocks: int) -> bool:
    if not x.is_cuda:
        return False
    B, H, W, C = (int(d) for d in x.shape)
    return (H, C // int(num_blocks)) in AFNO_FUSED_SHAPES


def afno_spectral_h(xw: torch.Tensor, w1, b1, w2, b2, num_blocks: int, lam: float, owner=None) -> torch.Tensor:
    """Fused H-filter on the W half spectrum ``xw`` [B, H, KM, C, 2]: bf16 MFMA operands for a
    bf16 spectrum, the bf16x3 split GEMMs for an fp32 spectrum."""
    split = xw.dtype == torch.float32
    if owner is not None:
        packed = module_cached(owner, f"afno_w{'3' if split else ''}", (w1, b1, w2, b2),
                               lambda: pack_afno_weights(w1, b1, w2, b2, split))
    else:
        packed = pack_afno_weights(w1, b1, w2, b2, split)
    w1t, w2t, b1p, b2p = packed
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
    """fc + exact (erf) GELU through ATen: the generic-shape fallback of :func:`afno_block_mlp`
    (counted by ``note_fallback``; the fused blocks run the hand MFMA GEMM with the GELU in its
    epilogue)."""
    return F.gelu(F.linear(y2, fc.weight, fc.bias))


class LnCarry(NamedTuple):
    """A per-channel pending bias plus the next LayerNorm's statistics of ``x + bias`` as
    per-64-channel partials (``linear3_stats`` / ``linear_stats``), carried from one block to the next."""
    bias: torch.Tensor
    part: torch.Tensor


class SplitRows(NamedTuple):
    """A block output already in the bf16x3 pair-row layout [tokens, 2C] (the last fp32 block
    writes the head GEMM's operand straight from its fc2 epilogue)."""
    pairs: torch.Tensor


def pending_bias(pending):
    """The residual-stream tensor part of a block's ``pending`` (drops carried statistics)."""
    return pending.bias if isinstance(pending, LnCarry) else pending


def afno_block_amd(blk, x: torch.Tensor, pending=None, split_out: bool = False):
    """One FourCastNet block on the MI355X path.

    Residual-stream fusion: the block returns ``(x, p)`` with the true block output being
    ``x + p``.  ``p`` is either a per-channel vector (the fc2 bias; LayerNorm-fused paths, see
    :func:`afno_block_fused` / :func:`afno_block_fused_f32`), an :class:`LnCarry` (that vector
    plus the next LayerNorm's partial statistics, LN-fused paths), or a full tensor (the fc2 output;
    generic path, where the addition is fused into the next block's LN1).
    ``split_out`` (last block before the fp32 head): the fp32 fused path may return its output as
    :class:`SplitRows` instead of an fp32 tensor.
    """
    part = None
    if isinstance(pending, LnCarry):
        pending, part = pending.bias, pending.part
    if pending is not None and pending.dim() == 1 and not _ln_fused_ok(blk, x):
        x, pending, part = x + pending, None, None
    if (pending is None or pending.dim() == 1) and _ln_fused_ok(blk, x):
        if x.dtype == torch.float32:
            return afno_block_fused_f32(blk, x, pending, part, split_out)
        return afno_block_fused(blk, x, pending, part)
    x, yn = afno_block_spectral(blk, x, pending)
    return x, afno_block_mlp(blk, yn)


def _f32(owner, name: str, t: torch.Tensor) -> torch.Tensor:
    """fp32 contiguous copy of a small parameter, cached on its module (capture safe)."""
    return module_cached(owner, name, (t,), lambda: t.detach().float().contiguous())


def _ln_fused_ok(blk, x: torch.Tensor) -> bool:
    from ..models.afno import kept_window

    f = blk.filter
    c = f.cfg
    if not (x.is_cuda and x.dtype in (torch.bfloat16, torch.float32) and x.dim() == 4 and x.shape[-1] % 8 == 0):
        return False
    B, H, W, C = (int(d) for d in x.shape)
    r0, r1, km = kept_window(H, W, c.hard_thresholding_fraction)
    if not _mlp_gemm_ok(blk.mlp, x.dtype == torch.float32):
        return False
    return r0 == 0 and r1 == H and afno_fused_available(x, c.num_blocks)


def _mlp_gemm_ok(m, split: bool) -> bool:
    """Both MLP GEMMs fit the hand kernel (csrc/nn/gemm.hip): output features in 64-feature
    halves (a ragged last 256-feature panel is masked in the kernel) and the reduction depth in
    64-tiles (bf16) or 32-tiles of at least 64 (bf16x3 split)."""
    def k_ok(k: int) -> bool:
        return k % 32 == 0 and k >= 64 if split else k % 64 == 0

    f1, f2 = m.fc1, m.fc2
    return (f1.out_features % 64 == 0 and f2.out_features % 64 == 0 and k_ok(f1.in_features)
            and k_ok(f2.in_features))


# AFNOConfig.bf16_gelu -> the hand GEMM's epilogue activation for bf16 outputs (csrc/nn/gelu.h):
#   "erf"       the erf GELU as x sigmoid(x q(x^2)), |error| <= 2.6e-5 absolute against the exact form
#               (1/40 of half a bf16 ulp at |y| = 0.25) -- FourCastNet's nn.GELU at bf16 resolution
#   "erf_exact" the A&S 7.1.26 erf form the fp32 path uses (|error| <= 1.5e-7)
#   "tanh"      torch's approximate="tanh" (|difference| <= 4.7e-4: an explicit opt-in)
_BF16_GELU_ACT = {"erf": 3, "erf_exact": 1, "tanh": 2}


def afno_block_fused(blk, xs: torch.Tensor, pre: Optional[torch.Tensor] = None, part: Optional[torch.Tensor] = None):
    """FourCastNet block (bf16) with LN1 fused into the AFNO W-transforms and fc2 accumulated
    in place.

    The residual stream is carried as ``(xs, pre)`` with true x = xs + pre (pre = the previous
    block's fc2 bias, per channel, or None):

      stats = (mean, rstd) of x                  ln_stats_merge of the previous fc2's partials
                                                 (first block: ln_stats over xs)
      X_w   = R2C_W(LN1(x))                      LN applied on load (no normalised copy in HBM)
      Y_w   = FFT_H -> block MLP -> IFFT_H       afno_spectral (MFMA)
      x1    = C2R_W(Y_w) + LN1(x) + x            both skips from one read of xs; the epilogue also
                                                 writes LN2's per-64-channel partials of the stored
                                                 x1 (c2r_ln_add_part)
      h     = GELU(fc1(LN2(x1)))                 ln_stats_merge + hand MFMA GEMM with LN2 folded in
                                                 (linear_ln) and the GELU in the epilogue -- FourCastNet's
                                                 erf form at bf16-output resolution unless cfg.bf16_gelu says
                                                 otherwise (see AFNOConfig and _BF16_GELU_ACT)
      x1   += h @ W2^T                           hand MFMA GEMM, residual in the epilogue, which also
                                                 emits the next LN1's partials of x1 + b2
                                                 (linear_stats)

    ``part``: those partials from the previous block (else ln_stats runs).  Returns
    (x1, LnCarry(fc2.bias, partials)): the bias is folded into the next block's statistics and
    loads (or the head GEMM's bias).  No pass over the residual stream beyond the block's own
    kernels (round 3: two ln_stats passes per block, 0.28 ms of 6.3).
    """
    from ..models.afno import kept_window

    f = blk.filter
    c = f.cfg
    n1 = blk.norm1
    B, H, W, C = (int(d) for d in xs.shape)  # static ints (constants under tracing)
    _, _, km = kept_window(H, W, c.hard_thresholding_fraction)
    scale = 1.0 / math.sqrt(H * W)
    ops = _ops()
    m = blk.mlp
    pre32 = None if pre is None else _f32(blk, "pre", pre)
    g1, be1 = _f32(blk, "g1", n1.weight), _f32(blk, "b1", n1.bias)
    stats = ops.ln_stats_merge(part, n1.eps) if part is not None else ops.ln_stats(xs, pre32, n1.eps)
    xw = ops.r2c_ln(xs, 2, scale, km, stats, g1, be1, pre32, torch.bfloat16)
    yw = afno_spectral_h(xw, f.w1, f.b1, f.w2, f.b2, c.num_blocks, c.sparsity_threshold, owner=f)
    # hand MFMA GEMM (csrc/nn/gemm.hip): one workgroup per output tile, no cross-workgroup
    # dependencies -- unaffected by long-lived kernels of other streams/processes (RCCL collective
    # blocks).  LN2 is folded into fc1 (linear_ln): only the per-token statistics, merged from the
    # C2R epilogue's partials (ln_stats_merge takes <= 64 chunks of 64 channels).
    if C <= 64 * 64:
        x1, part2 = ops.c2r_ln_add_part(yw, 2, W, scale, xs, stats, g1, be1, pre32)
        st2 = ops.ln_stats_merge(part2, blk.norm2.eps)
    else:
        x1 = ops.c2r_ln_add(yw, 2, W, scale, xs, stats, g1, be1, pre32)
        st2 = ops.ln_stats(x1, None, blk.norm2.eps)
    w1g, c1, c2 = _ln_folded_fc(m.fc1, blk.norm2)
    hid = ops.linear_ln(x1.reshape(-1, C), w1g, c1, c2, st2, _BF16_GELU_ACT[getattr(c, "bf16_gelu", "erf")])
    if C > 64 * 64:
        x1 = ops.linear(hid, m.fc2.weight, None, 0, x1.reshape(-1, C)).reshape(B, H, W, C)
        return x1, m.fc2.bias
    b2 = _f32(m, "fc2_b", m.fc2.bias)
    x1n, part_next = ops.linear_stats(hid, m.fc2.weight, x1.reshape(-1, C), b2)
    return x1n.reshape(B, H, W, C), LnCarry(m.fc2.bias, part_next)


def _ln_folded_fc(fc: torch.nn.Linear, ln: torch.nn.LayerNorm):
    """(W * gamma as bf16, c1 = row sums of that bf16 matrix, c2 = W beta + b): the operands of
    ``linear_ln`` for fc(LN(x)), cached on the Linear module."""
    def build():
        w = fc.weight.float()
        wg = (w * ln.weight.float()[None, :]).to(torch.bfloat16).contiguous()
        c1 = wg.float().sum(1).contiguous()
        c2 = (w @ ln.bias.float() + (fc.bias.float() if fc.bias is not None else 0.0)).contiguous()
        return wg, c1, c2

    return module_cached(fc, "ln_folded", (fc.weight, ln.weight, ln.bias) + ((fc.bias,) if fc.bias is not None else ()),
                         build)


def _ln_folded_fc3(fc: torch.nn.Linear, ln: torch.nn.LayerNorm):
    """fc(LN(x)) with the LayerNorm folded, bf16x3 operands: (split(W * gamma), c1, c2) with
    c1[n] = sum_k (hi + lo)[n, k] of exactly the split pairs the GEMM reads (so the mean term
    cancels the GEMM's own representation of W * gamma) and c2 = W beta + b, both summed in fp64.
    Cached on the Linear module."""
    def build():
        w = fc.weight.double()
        ws = split_bf16((w * ln.weight.double()[None, :]).float())
        c1 = unsplit_bf16(ws).double().sum(1).float().contiguous()
        c2 = w @ ln.bias.double()
        if fc.bias is not None:
            c2 = c2 + fc.bias.double()
        return ws, c1, c2.float().contiguous()

    return module_cached(fc, "ln_folded3", (fc.weight, ln.weight, ln.bias) + ((fc.bias,) if fc.bias is not None else ()),
                         build)


def afno_block_fused_f32(blk, xs: torch.Tensor, pre: Optional[torch.Tensor] = None, part: Optional[torch.Tensor] = None,
                         split_out: bool = False, residual_mode: str = "fp32"):
    """FourCastNet block at fp32 (the reference precision), every step on a hand kernel:

      stats = (mean, rstd) of x                  ln_stats_merge of the previous fc2's partials
                                                 (first block: ln_stats over x)
      X_w   = R2C_W(LN1(x))                      afno_wfft fp32 instantiation, fp32 spectrum
      Y_w   = FFT_H -> block MLP -> IFFT_H       afno_spectral bf16x3 variant (fp32 staging)
      x1    = C2R_W(Y_w) + LN1(x) + x            afno_wfft fp32, whose epilogue ALSO writes the
                                                 bf16x3 split pairs of x1 - mean(x) (centred per
                                                 token) and LN2's per-64-channel partials
                                                 (c2r_ln_add_split: no LayerNorm / split pass)
      st2   = (mean - mean(x), rstd) of x1       ln_stats_merge(shift=stats) (8 B per token)
      h     = split(GELU(LN2(x1) W1^T + b1))     bf16x3 GEMM on x1's pairs with LN2 folded into the
                                                 epilogue (linear3_ln), erf GELU, split-pair output
      x1    = x1 + h W2^T                        bf16x3 GEMM, fp32 residual epilogue, which also
                                                 emits the next LN1's statistics of x1 + b2 as
                                                 per-64-channel partials

    ``part``: those partials from the previous block (else ln_stats runs).  Returns
    (x1, LnCarry(fc2.bias, partials)); with ``split_out`` (last block) fc2 writes x1 as bf16x3
    pair rows for the head GEMM instead (no statistics, no separate split pass): (SplitRows, fc2.bias).

    ``residual_mode`` -- how x1 reaches fc2's residual epilogue (profiles/f32_pair_residual_r5.txt):
    "fp32" (what the model runs) the C2R epilogue's fp32 copy of x1; "pairs" the split pairs fc1
    reads + the per-token LN1 mean (full-depth rel-L2 1.0e-5 instead of 6.4e-6); "lo2" the pairs + a
    bf16 third term.  The two alternatives were measured and not adopted; they stay reachable by
    calling this function directly (tests, bench scripts), not through any global switch."""
    from ..models.afno import kept_window

    f = blk.filter
    c = f.cfg
    n1, n2, m = blk.norm1, blk.norm2, blk.mlp
    B, H, W, C = (int(d) for d in xs.shape)  # static ints (constants under tracing)
    _, _, km = kept_window(H, W, c.hard_thresholding_fraction)
    scale = 1.0 / math.sqrt(H * W)
    ops = _ops()
    pre32 = None if pre is None else _f32(blk, "pre", pre)
    g1, be1 = _f32(blk, "g1", n1.weight), _f32(blk, "b1", n1.bias)
    stats = ops.ln_stats_merge(part, n1.eps) if part is not None else ops.ln_stats(xs, pre32, n1.eps)
    xw = ops.r2c_ln(xs, 2, scale, km, stats, g1, be1, pre32, torch.float32)
    yw = afno_spectral_h(xw, f.w1, f.b1, f.w2, f.b2, c.num_blocks, c.sparsity_threshold, owner=f)
    # "pairs" / "lo2": fc2 takes the residual as x1's split pairs (+ the per-token shift, + the third
    # term), so the C2R epilogue skips x1's fp32 copy -- the largest of its output streams
    if residual_mode not in ("fp32", "pairs", "lo2"):
        raise ValueError(f"residual_mode must be 'fp32', 'pairs' or 'lo2', got {residual_mode!r}")
    mode = residual_mode if (not split_out and C <= 64 * 64) else "fp32"
    x1, x1s, part2 = ops.c2r_ln_add_split(yw, 2, W, scale, xs, stats, g1, be1, pre32,
                                          {"fp32": 1, "pairs": 0, "lo2": 2}[mode])
    # x1s holds x1 - mean(x) per token (centred split): st2's mean is shifted to match.
    # ln_stats_merge takes <= 64 chunks of 64 channels
    if C <= 64 * 64:
        st2 = ops.ln_stats_merge(part2, n2.eps, stats)
    else:
        st2 = ops.ln_stats(x1, None, n2.eps)
        st2 = torch.stack((st2[:, 0] - stats.reshape(-1, 2)[:, 0], st2[:, 1]), 1)
    w1s, c1, c2 = _ln_folded_fc3(m.fc1, n2)
    hid = ops.linear3_ln(x1s, w1s, c1, c2, st2, 1)
    w2s = module_cached(m, "fc2_split", (m.fc2.weight,), lambda: split_bf16(m.fc2.weight))
    if split_out:
        return SplitRows(ops.linear3(hid, w2s, None, 0, x1.reshape(-1, C), True)), m.fc2.bias
    if C > 64 * 64:  # ln_stats_merge takes <= 64 chunks of 64 channels
        x1 = ops.linear3(hid, w2s, None, 0, x1.reshape(-1, C), False).reshape(B, H, W, C)
        return x1, m.fc2.bias
    b2 = _f32(m, "fc2_b", m.fc2.bias)
    if mode != "fp32":
        x1n, part_next = ops.linear3_stats_pr(hid, w2s, x1s, stats.reshape(-1, 2), b2, x1 if mode == "lo2" else None)
    else:
        x1n, part_next = ops.linear3_stats(hid, w2s, x1.reshape(-1, C), b2)
    return x1n.reshape(B, H, W, C), LnCarry(m.fc2.bias, part_next)


def afno_block_spectral(blk, x: torch.Tensor, pending: Optional[torch.Tensor] = None):
    """Bandwidth/VALU-bound half of a block: LN1(+pending residual) -> AFNO filter (+ both skips,
    fused into the C2R store) -> LN2.  Returns (residual stream x, LN2 output)."""
    from ..models.afno import afno2d_amd

    f = blk.filter
    c = f.cfg
    h, x = _ops().layer_norm(x, blk.norm1.weight, blk.norm1.bias, blk.norm1.eps, pending)
    # filter(LN1(x)) + LN1(x) [AFNO bias] + x [double skip], fused into the C2R store
    x = afno2d_amd(h, f.w1, f.b1, f.w2, f.b2, c.num_blocks, c.sparsity_threshold, c.hard_thresholding_fraction,
                   residual=x, owner=f)
    yn, _ = layer_norm(x, blk.norm2)
    return x, yn


def afno_block_mlp(blk, yn: torch.Tensor) -> torch.Tensor:
    """MFMA-bound half of a block (generic shapes): fc1 + GELU and fc2 + bias."""
    m = blk.mlp
    B, H, W, C = yn.shape
    # the generic-shape path leaves the hand GEMM: counted (fallback_counts, MI_DFT_STRICT).  Under
    # hipGraph capture a note fires once per captured call, not per replay.
    note_fallback("mlp_fc1_gelu", "hipBLASLt / ATen fc1+GELU instead of the hand MFMA GEMM", yn)
    hid = _gelu_linear(yn.reshape(-1, C), m.fc1)
    note_fallback("mlp_fc2", "ATen / hipBLASLt fc2 (generic AFNO shape)", yn)
    y = F.linear(hid, m.fc2.weight, m.fc2.bias)
    return y.reshape(B, H, W, C)


def fno_spectral_mix(xm: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """FNO mode mixing out[b,o,m] = sum_i x[b,i,m] w[i,o,m] on complex-as-pair tensors
    xm [B, Cin, M, 2], w [Cin, Cout, M, 2] -> [B, Cout, M, 2] (fp32).  Native op on every device
    (CPU: ATen einsum; GPU: csrc/spectral/fno_mix.hip), so it also exports as one ONNX node."""
    return _ops().fno_mix(xm.contiguous(), w.contiguous())
