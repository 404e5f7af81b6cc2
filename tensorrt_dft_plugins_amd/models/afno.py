"""FourCastNet AFNO network (Adaptive Fourier Neural Operator), random-initialised.

The reference names FourCastNet only as its motivating workload (/root/reference/README.md:3);
the architecture here follows the public FourCastNet AFNO design (Pathak et al. 2022):
patch-embed (8x8 conv, 20 -> 768) + positional embedding, 12 blocks of
[LayerNorm -> AFNO2D spectral filter -> (+residual, double skip) -> LayerNorm -> MLP(4x, GELU)
-> +residual], linear head 768 -> 20*8*8 and un-patchify to [B, 20, 720, 1440].

AFNO2D: rfft2 over (H, W) of the channel-last tokens (norm="ortho"); a block-diagonal
2-layer complex MLP (8 blocks of 96 channels, ReLU, bias) on the kept modes
(all H rows x the first ``H//2+1`` W-modes at hard_thresholding_fraction=1, exactly FourCastNet's
slicing), softshrink(0.01), irfft2, + the filter input.

Backends:
* ``"torch"``  -- plain PyTorch (torch.fft, einsum): the numerics oracle and eager comparator.
* ``"contrib"`` -- the same network written the reference's way: the FFTs are the ONNX-contrib
  ``OnnxRfft2`` / ``OnnxIrfft2`` Functions (/root/reference/tests/test_dft.py:35-60) around a
  channel-last permute, so it exports to a stock ONNX graph (Rfft / Irfft + einsums, LayerNorms,
  MatMuls) that the engine's build-time rewrite pass (``onnx/optimizer.py``) maps onto the hand
  kernels.
* ``"amd"``    -- MI355X path: pruned hand-written FFTs (only kept modes are computed),
  fused spectral-MLP kernel (MFMA), fused LayerNorm, bf16 GEMMs.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import dft as D
from ..utils.trace import trace_range


@dataclass
class AFNOConfig:
    img_size: Tuple[int, int] = (720, 1440)
    patch_size: int = 8
    in_chans: int = 20
    out_chans: int = 20
    embed_dim: int = 768
    depth: int = 12
    mlp_ratio: float = 4.0
    num_blocks: int = 8
    sparsity_threshold: float = 0.01
    hard_thresholding_fraction: float = 1.0
    # GELU of the bf16 block's fc1 epilogue on the hand GEMM (ops.spectral._BF16_GELU_ACT):
    #   "erf" (default) FourCastNet's nn.GELU, evaluated as x sigmoid(x q(x^2)) to 2.6e-5 absolute of
    #         the exact form -- below bf16 output resolution, at about the tanh form's cost;
    #   "erf_exact" the A&S erf form of the fp32 path; "tanh" torch's approximate="tanh" (|difference|
    #         <= 4.7e-4, an explicit opt-in; profiles/gelu_tanh_bf16_r5.txt).
    # fp32 models always use the exact erf form.
    bf16_gelu: str = "erf"

    @property
    def h(self) -> int:
        return self.img_size[0] // self.patch_size

    @property
    def w(self) -> int:
        return self.img_size[1] // self.patch_size


def fourcastnet_config(**kw) -> AFNOConfig:
    """FourCastNet (ERA5 0.25 deg, 20 variables) hyper-parameters."""
    return AFNOConfig(**kw)


def afno2d_reference(x, w1, b1, w2, b2, num_blocks, sparsity_threshold, hard_thresholding_fraction):
    """FourCastNet AFNO2D forward in plain PyTorch (fp32 FFT), used as the oracle."""
    bias = x
    dtype = x.dtype
    x = x.float()
    B, H, W, C = x.shape
    bs = C // num_blocks
    x = torch.fft.rfft2(x, dim=(1, 2), norm="ortho")
    x = x.reshape(B, H, W // 2 + 1, num_blocks, bs)
    total_modes = H // 2 + 1
    kept = int(total_modes * hard_thresholding_fraction)
    rs = slice(total_modes - kept, total_modes + kept)
    xs = x[:, rs, :kept]
    o1r = F.relu(torch.einsum("...bi,bio->...bo", xs.real, w1[0]) - torch.einsum("...bi,bio->...bo", xs.imag, w1[1]) + b1[0])
    o1i = F.relu(torch.einsum("...bi,bio->...bo", xs.imag, w1[0]) + torch.einsum("...bi,bio->...bo", xs.real, w1[1]) + b1[1])
    o2r = torch.einsum("...bi,bio->...bo", o1r, w2[0]) - torch.einsum("...bi,bio->...bo", o1i, w2[1]) + b2[0]
    o2i = torch.einsum("...bi,bio->...bo", o1i, w2[0]) + torch.einsum("...bi,bio->...bo", o1r, w2[1]) + b2[1]
    o2 = torch.zeros(B, H, W // 2 + 1, num_blocks, bs, 2, device=x.device)
    o2[:, rs, :kept] = torch.stack([o2r, o2i], dim=-1)
    o2 = F.softshrink(o2, lambd=sparsity_threshold)
    x = torch.view_as_complex(o2).reshape(B, H, W // 2 + 1, C)
    x = torch.fft.irfft2(x, s=(H, W), dim=(1, 2), norm="ortho")
    return x.type(dtype) + bias


def afno2d_contrib(x, w1, b1, w2, b2, num_blocks, sparsity_threshold, hard_thresholding_fraction):
    """FourCastNet AFNO2D with the ONNX-contrib DFT ops (exportable the reference's way).

    ``Rfft`` / ``Irfft`` transform the LAST two dims with the "backward" norm (the contrib
    contract), so the channel-last tokens are permuted to [B, C, H, W] around them and the ortho
    scales are explicit multiplies; the kept-mode window is sliced out, run through the
    block-diagonal complex MLP as real/imaginary einsums, softshrunk and zero-padded back."""
    from ..onnx.exporter import OnnxIrfft2, OnnxRfft2

    bias = x
    B, H, W, C = (int(d) for d in x.shape)
    nb = int(num_blocks)
    bs = C // nb
    wf = W // 2 + 1
    r0, r1, km = kept_window(H, W, hard_thresholding_fraction)
    X = OnnxRfft2.apply(x.float().permute(0, 3, 1, 2)) * (1.0 / math.sqrt(H * W))  # [B, C, H, wf, 2], ortho
    X = X.permute(0, 2, 3, 1, 4)[:, r0:r1, :km].reshape(B, r1 - r0, km, nb, bs, 2)
    xr, xi = X[..., 0], X[..., 1]
    o1r = F.relu(torch.einsum("...bi,bio->...bo", xr, w1[0]) - torch.einsum("...bi,bio->...bo", xi, w1[1]) + b1[0])
    o1i = F.relu(torch.einsum("...bi,bio->...bo", xi, w1[0]) + torch.einsum("...bi,bio->...bo", xr, w1[1]) + b1[1])
    o2r = torch.einsum("...bi,bio->...bo", o1r, w2[0]) - torch.einsum("...bi,bio->...bo", o1i, w2[1]) + b2[0]
    o2i = torch.einsum("...bi,bio->...bo", o1i, w2[0]) + torch.einsum("...bi,bio->...bo", o1r, w2[1]) + b2[1]
    o2 = F.softshrink(torch.stack([o2r, o2i], dim=-1), lambd=sparsity_threshold).reshape(B, r1 - r0, km, C, 2)
    o2 = F.pad(o2, (0, 0, 0, 0, 0, wf - km, r0, H - r1))  # zero modes outside the window
    y = OnnxIrfft2.apply(o2.permute(0, 3, 1, 2, 4)) * math.sqrt(H * W)  # Irfft is 1/N: ortho = x sqrt(N)
    return y.permute(0, 2, 3, 1).to(x.dtype) + bias


def kept_window(H: int, W: int, fraction: float) -> Tuple[int, int, int]:
    """(row_start, row_stop, kept_w_modes) of FourCastNet's mode slicing."""
    total = H // 2 + 1
    kept = int(total * fraction)
    r0, r1 = max(0, total - kept), min(H, total + kept)
    return r0, r1, min(kept, W // 2 + 1)


class AFNO2D(nn.Module):
    def __init__(self, cfg: AFNOConfig, backend: str = "torch"):
        super().__init__()
        C = cfg.embed_dim
        self.cfg = cfg
        self.backend = backend
        self.num_blocks = cfg.num_blocks
        self.bs = C // cfg.num_blocks
        s = 0.02
        self.w1 = nn.Parameter(s * torch.randn(2, self.num_blocks, self.bs, self.bs))
        self.b1 = nn.Parameter(s * torch.randn(2, self.num_blocks, self.bs))
        self.w2 = nn.Parameter(s * torch.randn(2, self.num_blocks, self.bs, self.bs))
        self.b2 = nn.Parameter(s * torch.randn(2, self.num_blocks, self.bs))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        c = self.cfg
        if self.backend == "contrib":
            return afno2d_contrib(x, self.w1, self.b1, self.w2, self.b2, c.num_blocks, c.sparsity_threshold,
                                  c.hard_thresholding_fraction)
        if self.backend == "torch":
            return afno2d_reference(x, self.w1, self.b1, self.w2, self.b2, c.num_blocks, c.sparsity_threshold,
                                    c.hard_thresholding_fraction)
        return afno2d_amd(x, self.w1, self.b1, self.w2, self.b2, c.num_blocks, c.sparsity_threshold,
                          c.hard_thresholding_fraction, owner=self)


def afno2d_amd(x, w1, b1, w2, b2, num_blocks, sparsity_threshold, hard_thresholding_fraction, residual=None,
               owner=None):
    """MI355X AFNO2D: pruned R2C along W (only kept W-modes), fused [FFT_H -> block MLP ->
    softshrink -> IFFT_H] spectral kernel, pruned C2R along W with the filter bias fused.
    Falls back to pruned FFTs + torch GEMMs when the fused kernel does not apply."""
    from ..ops import spectral as S

    B, H, W, C = x.shape
    r0, r1, km = kept_window(H, W, hard_thresholding_fraction)
    scale_f = 1.0 / math.sqrt(H * W)
    if S.afno_fused_available(x, num_blocks) and r0 == 0 and r1 == H:
        # W-direction R2C keeping km modes: [B, H, km, C, 2] (bf16 for bf16 models: halves the
        # spectrum traffic; the spectral MLP consumes bf16 MFMA operands anyway; FFTs are fp32
        # in registers/LDS)
        sdt = torch.bfloat16 if x.dtype == torch.bfloat16 else torch.float32
        xw = D._ops().r2c(x, [2], scale_f, [km, 0], sdt)
        yw = S.afno_spectral_h(xw, w1, b1, w2, b2, num_blocks, sparsity_threshold, owner=owner)
        # C2R along W from km stored modes, + bias (filter input) fused
        return S.c2r_w_add(yw, x, W, 1.0 / math.sqrt(H * W), residual)
    # generic path: pruned 2-D R2C/C2R + batched real-block GEMMs
    S.note_fallback("afno_spectral", "no fused AFNO kernel for this (H, block size) / mode window: torch.baddbmm", x)
    xf = D._ops().r2c(x, [1, 2], scale_f, [H, 0, km, 0], torch.float32)[:, r0:r1]
    bs = C // num_blocks
    M = xf.shape[0] * xf.shape[1] * xf.shape[2]
    z = xf.reshape(M, num_blocks, bs, 2).permute(1, 0, 3, 2).reshape(num_blocks, M, 2 * bs)  # [nb, M, (re|im)*bs]
    w1, b1, w2, b2 = w1.float(), b1.float(), w2.float(), b2.float()  # fp32 spectrum math for any model dtype
    W1 = torch.cat([torch.cat([w1[0], w1[1]], dim=2), torch.cat([-w1[1], w1[0]], dim=2)], dim=1)  # [nb, 2bs, 2bs]
    W2 = torch.cat([torch.cat([w2[0], w2[1]], dim=2), torch.cat([-w2[1], w2[0]], dim=2)], dim=1)
    h = torch.relu(torch.baddbmm(torch.cat([b1[0], b1[1]], 1).unsqueeze(1), z, W1))
    o = torch.baddbmm(torch.cat([b2[0], b2[1]], 1).unsqueeze(1), h, W2)
    o = F.softshrink(o, sparsity_threshold)
    o = o.reshape(num_blocks, M, 2, bs).permute(1, 0, 3, 2).reshape(xf.shape[0], r1 - r0, km, C, 2)
    if r0 > 0 or r1 < H:
        full = o.new_zeros(o.shape[0], H, km, C, 2)
        full[:, r0:r1] = o
        o = full
    y = D._ops().c2r(o.contiguous(), [1, 2], [H, W], scale_f, [H, 0, km, 0], torch.float32)
    out = y.to(x.dtype) + x
    if residual is not None:
        out = out + residual
    return out


class Mlp(nn.Module):
    def __init__(self, dim: int, hidden: int):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)

    def forward(self, x):
        return self.fc2(F.gelu(self.fc1(x)))


class Block(nn.Module):
    def __init__(self, cfg: AFNOConfig, backend: str = "torch"):
        super().__init__()
        self.backend = backend
        self.norm1 = nn.LayerNorm(cfg.embed_dim, eps=1e-6)
        self.filter = AFNO2D(cfg, backend)
        self.norm2 = nn.LayerNorm(cfg.embed_dim, eps=1e-6)
        self.mlp = Mlp(cfg.embed_dim, int(cfg.embed_dim * cfg.mlp_ratio))

    def forward(self, x):
        if self.backend == "amd":
            from ..ops import spectral as S

            x, y = S.afno_block_amd(self, x)
            return x + S.pending_bias(y)
        residual = x
        x = self.filter(self.norm1(x))
        x = x + residual  # double skip
        residual = x
        x = self.mlp(self.norm2(x))
        return x + residual


class AFNONet(nn.Module):
    """FourCastNet AFNO backbone.  Input [B, in_chans, H, W] -> output [B, out_chans, H, W]."""

    def __init__(self, cfg: Optional[AFNOConfig] = None, backend: str = "torch"):
        super().__init__()
        self.cfg = cfg = cfg or AFNOConfig()
        self.backend = backend
        p = cfg.patch_size
        self.patch_embed = nn.Conv2d(cfg.in_chans, cfg.embed_dim, kernel_size=p, stride=p)
        self.pos_embed = nn.Parameter(0.02 * torch.randn(1, cfg.h * cfg.w, cfg.embed_dim))
        self.blocks = nn.ModuleList([Block(cfg, backend) for _ in range(cfg.depth)])
        self.head = nn.Linear(cfg.embed_dim, cfg.out_chans * p * p, bias=False)

    def set_backend(self, backend: str) -> "AFNONet":
        self.backend = backend
        for b in self.blocks:
            b.backend = backend
            b.filter.backend = backend
        return self

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        cfg = self.cfg
        B = x.shape[0]
        p = cfg.patch_size
        f32 = self.backend == "amd" and x.is_cuda and x.dtype == torch.float32 and self._f32_native()
        if self.backend == "amd":
            from .._loader import load_plugins
            from ..ops import spectral as S

            load_plugins()
            # conv with kernel == stride is a GEMM over non-overlapping patches: one MFMA GEMM
            # gathers the 8x8 patches straight from the image, bias + position embedding in its
            # epilogue (no patchified copy, no separate add)
            pos = self.pos_embed.reshape(cfg.h * cfg.w, cfg.embed_dim)
            if f32:  # bf16x3: the raw fp32 image (split into bf16 planes by the op), split weights
                pe = self.patch_embed
                ws = S.module_cached(self, "embed_split", (pe.weight,),
                                     lambda: S.split_bf16(pe.weight.reshape(cfg.embed_dim, -1)))
                t = torch.ops.amd_dft.patch_linear3(x.contiguous(), ws, pe.bias, pos, p)
            else:
                wmat = self.patch_embed.weight.reshape(cfg.embed_dim, -1)
                t = torch.ops.amd_dft.patch_linear(x, wmat, self.patch_embed.bias, pos, p)
            t = t.reshape(B, cfg.h, cfg.w, cfg.embed_dim)
        else:
            t = self.patch_embed(x).flatten(2).transpose(1, 2)
            t = (t + self.pos_embed).reshape(B, cfg.h, cfg.w, cfg.embed_dim)
        if self.backend == "amd":
            from ..ops import spectral as S

            pending = None
            nblk = len(self.blocks)
            for i, blk in enumerate(self.blocks):
                with trace_range(f"afno.block{i}"):
                    t, pending = S.afno_block_amd(blk, t, pending, split_out=f32 and i == nblk - 1)
            hb = None
            pending = S.pending_bias(pending)  # the head needs no LayerNorm statistics
            if pending is not None and pending.dim() == 1:
                # per-channel residual bias left by the LN-fused blocks: folded into the
                # head GEMM's bias, head(t + p) = head(t) + W_head p
                hb = self._head_bias_cpp(pending)
            elif pending is not None:
                t = t + pending
            # head GEMM (features permuted to (c_out, p1, p2)) with the un-patchify folded into its
            # output scatter
            if f32:
                hw = self._head_weight_cpp()
                ws = S.module_cached(self, "head_split", (hw,), lambda: S.split_bf16(hw))
                ts = t.pairs if isinstance(t, S.SplitRows) else S.split_bf16(t.reshape(-1, cfg.embed_dim))
                return torch.ops.amd_dft.linear_unpatch3(ts, ws, hb, cfg.out_chans, cfg.h, cfg.w, p)
            tt = t.reshape(-1, cfg.embed_dim)
            return torch.ops.amd_dft.linear_unpatch(tt, self._head_weight_cpp(), hb, cfg.out_chans, cfg.h, cfg.w, p)
        for blk in self.blocks:
            t = blk(t)
        t = self.head(t)  # [B, h, w, out*p*p], feature order (p1, p2, c_out) as FourCastNet
        t = t.reshape(B, cfg.h, cfg.w, p, p, cfg.out_chans).permute(0, 5, 1, 3, 2, 4)
        return t.reshape(B, cfg.out_chans, cfg.h * p, cfg.w * p)

    def _f32_native(self) -> bool:
        """fp32 on the hand kernels (bf16x3 GEMMs) needs the embed/MLP/head widths in 64-feature
        halves (ragged 256-feature panels are masked in the GEMM) and 8x8 patches."""
        cfg = self.cfg
        hid = int(cfg.embed_dim * cfg.mlp_ratio)
        return (cfg.embed_dim % 64 == 0 and hid % 64 == 0 and (cfg.out_chans * cfg.patch_size ** 2) % 64 == 0
                and cfg.patch_size == 8)

    def _head_bias_cpp(self, pre: torch.Tensor) -> torch.Tensor:
        """W_head(c_out, p1, p2 order) @ pre as an fp32 bias, cached on the module."""
        from ..ops.spectral import module_cached

        w = self._head_weight_cpp()
        return module_cached(self, "head_bias", (w, pre), lambda: w.float() @ pre.float())

    def _head_weight_cpp(self) -> torch.Tensor:
        """Head weight with rows reordered from (p1, p2, c_out) to (c_out, p1, p2); cached."""
        from ..ops.spectral import module_cached

        w = self.head.weight
        p, co = self.cfg.patch_size, self.cfg.out_chans
        return module_cached(self, "head_weight", (w,),
                             lambda: w.reshape(p, p, co, -1).permute(2, 0, 1, 3).reshape(co * p * p, -1).contiguous())


def flops_per_sample(cfg: AFNOConfig) -> float:
    """Model FLOPs per sample (GEMMs + spectral MLP on the kept modes; FFTs excluded)."""
    N = cfg.h * cfg.w
    C = cfg.embed_dim
    hid = int(C * cfg.mlp_ratio)
    mlp = 2 * 2 * N * C * hid
    r0, r1, km = kept_window(cfg.h, cfg.w, cfg.hard_thresholding_fraction)
    modes = (r1 - r0) * km
    spec = modes * cfg.num_blocks * 2 * (2 * (2 * (C // cfg.num_blocks)) ** 2)
    embed = 2 * N * C * cfg.in_chans * cfg.patch_size ** 2
    head = 2 * N * C * cfg.out_chans * cfg.patch_size ** 2
    return cfg.depth * (mlp + spec) + embed + head
