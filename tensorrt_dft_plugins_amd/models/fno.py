"""Fourier Neural Operator (FNO, Li et al. 2021) on the MI355X DFT ops, random-initialised.

The reference's motivating workload is FNO-family models (/root/reference/README.md:3); its
TensorRT plugins supply the two FFT ends of every spectral layer
(/root/reference/src/dft_plugins.cpp:171-195 R2C/C2R exec), and the per-mode complex multiply
and the pointwise path run as ordinary TensorRT layers.  Here a spectral layer is three native
kernels per stage, and the full-resolution spectral output is never written to HBM:

  1. pruned R2C over (H, W): along W a truncated DFT on MFMA (``csrc/spectral/dft_gemm.hip``,
     only the kept ``[0, m2)`` modes), then a pruned Stockham FFT along H keeping
     ``[0, m1) u [H-m1, H)``;
  2. ``fno_mix_c2c`` -- the per-mode complex channel mixing computed in the first-pass gather of
     the pruned inverse FFT along H (the mixed modes are never stored; ``fno_mix`` on MFMA,
     ``csrc/spectral/fno_mix.hip``, plus ``c2c_axis`` where no fixed column kernel covers H);
  3. ``fno_c2r_pw``: the inverse truncated DFT
     along W on MFMA fused with the 1x1 convolution, bias and GELU
     (``csrc/spectral/fno_c2r_pw.hip``) -- reads x, writes y, nothing else; ``SpectralConv2d`` on its
     own ends with ``fno_c2r``, the same kernel without the pointwise branch (writes y only).

Backends: ``"torch"`` (torch.fft + einsum + conv2d, the numerics oracle), ``"contrib"`` (the same
layer written the reference's way: ONNX-contrib ``OnnxRfft2`` / ``OnnxIrfft2`` + real/imaginary
einsums + zero padding, /root/reference/tests/test_dft.py:35-60, exportable to a stock ONNX graph
that the engine's rewrite pass maps back onto the kernels below) and ``"amd"``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


__all__ = ["FNOConfig", "SpectralConv2d", "FNOBlock", "FNO2d", "spectral_conv2d_reference", "spectral_conv2d_contrib"]


@dataclass
class FNOConfig:
    img_size: Tuple[int, int] = (720, 1440)
    in_chans: int = 20
    out_chans: int = 20
    width: int = 20
    modes1: int = 32  # kept H modes on each side (low and high)
    modes2: int = 32  # kept W modes (one-sided)
    n_layers: int = 4
    proj_hidden: int = 128


def spectral_conv2d_reference(x: torch.Tensor, weight: torch.Tensor, m1: int, m2: int) -> torch.Tensor:
    """Classic FNO SpectralConv2d in plain PyTorch (fp32 FFT).

    ``weight``: [Cin, Cout, 2*m1, m2, 2] real, rows ``[0, m1)`` act on the low H modes and rows
    ``[m1, 2*m1)`` on the high (negative-frequency) H modes (the classic ``weights1/weights2``).
    """
    B, _, H, W = x.shape
    cout = weight.shape[1]
    wc = torch.view_as_complex(weight.float().contiguous())
    xf = torch.fft.rfft2(x.float())
    out = torch.zeros(B, cout, H, W // 2 + 1, dtype=torch.complex64, device=x.device)
    out[:, :, :m1, :m2] = torch.einsum("bixy,ioxy->boxy", xf[:, :, :m1, :m2], wc[:, :, :m1])
    out[:, :, H - m1:, :m2] = torch.einsum("bixy,ioxy->boxy", xf[:, :, H - m1:, :m2], wc[:, :, m1:])
    return torch.fft.irfft2(out, s=(H, W))


def spectral_conv2d_contrib(x: torch.Tensor, weight: torch.Tensor, m1: int, m2: int) -> torch.Tensor:
    """Classic FNO SpectralConv2d with the ONNX-contrib DFT ops: Rfft -> two mode windows ->
    complex channel mixing as real einsums -> zero padding -> Irfft (all "backward" norm)."""
    from ..onnx.exporter import OnnxIrfft2, OnnxRfft2

    B, _, H, W = (int(d) for d in x.shape)
    wf = W // 2 + 1
    X = OnnxRfft2.apply(x.float())  # [B, Cin, H, wf, 2]
    wr, wi = weight[..., 0].float(), weight[..., 1].float()

    def mix(xs, lo, hi):
        a, b = xs[..., 0], xs[..., 1]
        re = torch.einsum("bixy,ioxy->boxy", a, wr[:, :, lo:hi]) - torch.einsum("bixy,ioxy->boxy", b, wi[:, :, lo:hi])
        im = torch.einsum("bixy,ioxy->boxy", a, wi[:, :, lo:hi]) + torch.einsum("bixy,ioxy->boxy", b, wr[:, :, lo:hi])
        return torch.stack([re, im], dim=-1)

    top = F.pad(mix(X[:, :, :m1, :m2], 0, m1), (0, 0, 0, wf - m2, 0, H - m1))
    bot = F.pad(mix(X[:, :, H - m1:, :m2], m1, 2 * m1), (0, 0, 0, wf - m2, H - m1, 0))
    return OnnxIrfft2.apply(top + bot)


class SpectralConv2d(nn.Module):
    def __init__(self, in_ch: int, out_ch: int, modes1: int, modes2: int, backend: str = "torch"):
        super().__init__()
        self.in_ch, self.out_ch, self.modes1, self.modes2 = in_ch, out_ch, modes1, modes2
        self.backend = backend
        scale = 1.0 / (in_ch * out_ch)
        self.weight = nn.Parameter(scale * torch.rand(in_ch, out_ch, 2 * modes1, modes2, 2))

    def _check(self, H: int, W: int):
        if 2 * self.modes1 > H or self.modes2 > W // 2 + 1:
            raise ValueError(f"modes ({self.modes1}, {self.modes2}) do not fit a {H}x{W} grid")

    def spectrum(self, x: torch.Tensor) -> torch.Tensor:
        """Spectral path only: irfft2(mix(rfft2(x)))  ->  [B, Cout, H, W] in x.dtype (amd) / fp32 (torch)."""
        B, C, H, W = x.shape
        self._check(H, W)
        m1, m2 = self.modes1, self.modes2
        if self.backend == "torch":
            return spectral_conv2d_reference(x, self.weight, m1, m2)
        if self.backend == "contrib":
            return spectral_conv2d_contrib(x, self.weight, m1, m2)
        # FNOBlock's kernels without the pointwise branch: truncated DFT along W on MFMA, pruned FFT
        # along H, mixing inside the pruned inverse H transform, inverse truncated DFT along W (fno_c2r:
        # the layer tail with no x read) -- the full-resolution spectrum never exists
        ops = torch.ops.amd_dft
        xw = ops.dftw_r2c(x, m2, 1.0)  # [B, Cin, H, m2, 2]
        xm = ops.c2c_axis(xw, 2, H, H, 0, m1, m1, False, 1.0)  # [B, Cin, 2*m1, m2, 2]
        yw = ops.fno_mix_c2c(xm, self._packed_weight(), H, m1, m1, 1.0 / (H * W), 0)  # [B, Cout, H, m2, 2]
        out_dt = x.dtype if x.dtype in (torch.float32, torch.bfloat16) else torch.float32
        return ops.fno_c2r(yw, W, out_dt)

    def _packed_weight(self) -> torch.Tensor:
        w = self.weight
        if w.dtype != torch.float32:
            w = w.float()
        return w.reshape(self.in_ch, self.out_ch, 2 * self.modes1 * self.modes2, 2)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.spectrum(x)


class FNOBlock(nn.Module):
    """One FNO layer: ``act(SpectralConv2d(x) + Conv1x1(x))`` -- the "FNO SpectralConv2d block"."""

    def __init__(self, width: int, modes1: int, modes2: int, activation: bool = True, backend: str = "torch"):
        super().__init__()
        self.spectral = SpectralConv2d(width, width, modes1, modes2, backend)
        self.w = nn.Conv2d(width, width, 1)
        self.activation = activation
        self.backend = backend
        # mode-mixing path of the amd backend: 0 = by batch size (the native op's rule), 1 = inside
        # the inverse H transform's gather, 2 = batched MFMA GEMM (weights read once per batch)
        self.mix_path = 0

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.backend == "amd":
            return self._forward_amd(x)
        y = self.spectral(x).to(x.dtype) + self.w(x)
        return F.gelu(y) if self.activation else y

    def _forward_amd(self, x: torch.Tensor) -> torch.Tensor:
        """pruned R2C (MFMA DFT-GEMM along W + pruned FFT along H) -> [mode mixing + pruned inverse
        FFT along H] -> fused [inverse DFT-GEMM along W + 1x1 conv + bias + GELU]: four kernels.
        From batch 8 the mixing runs as batched per-mode GEMMs on MFMA (fno_mix.hip: every mode's
        weights read once for the whole batch) followed by the pruned inverse transform: five."""
        sp = self.spectral
        B, C, H, W = x.shape
        sp._check(H, W)
        m1, m2 = sp.modes1, sp.modes2
        ops = torch.ops.amd_dft
        xw = ops.dftw_r2c(x, m2, 1.0)  # [B, Cin, H, m2, 2]  truncated DFT along W on MFMA
        xm = ops.c2c_axis(xw, 2, H, H, 0, m1, m1, False, 1.0)  # [B, Cin, 2*m1, m2, 2]
        # mode mixing inside the inverse H transform's gather (one kernel; fno_mix + c2c_axis
        # where no fixed column kernel covers H)
        yw = ops.fno_mix_c2c(xm, sp._packed_weight(), H, m1, m1, 1.0 / (H * W), self.mix_path)  # [B, Cout, H, m2, 2]
        return ops.fno_c2r_pw(yw, x, self.w.weight.reshape(self.w.out_channels, -1).float(), self.w.bias.float(),
                              self.activation)


class FNO2d(nn.Module):
    """Lifting (1x1, in -> width) -> n_layers FNO blocks (last without activation) ->
    projection (1x1 width -> proj_hidden, GELU, 1x1 -> out)."""

    def __init__(self, cfg: Optional[FNOConfig] = None, backend: str = "torch"):
        super().__init__()
        self.cfg = cfg = cfg or FNOConfig()
        self.lift = nn.Conv2d(cfg.in_chans, cfg.width, 1)
        self.blocks = nn.ModuleList(
            [FNOBlock(cfg.width, cfg.modes1, cfg.modes2, activation=i < cfg.n_layers - 1, backend=backend)
             for i in range(cfg.n_layers)])
        self.proj1 = nn.Conv2d(cfg.width, cfg.proj_hidden, 1)
        self.proj2 = nn.Conv2d(cfg.proj_hidden, cfg.out_chans, 1)
        self.set_backend(backend)

    def set_backend(self, backend: str) -> "FNO2d":
        self.backend = backend
        for b in self.blocks:
            b.backend = backend
            b.spectral.backend = backend
        return self

    def _pw(self, conv: nn.Conv2d, x: torch.Tensor, gelu: bool) -> torch.Tensor:
        if self.backend == "amd":
            return torch.ops.amd_dft.fno_pointwise(None, x, conv.weight.float(), conv.bias.float(), gelu)
        y = conv(x)
        return F.gelu(y) if gelu else y

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.backend == "amd":
            from .._loader import load_plugins

            load_plugins()
        x = self._pw(self.lift, x, False)
        for b in self.blocks:
            x = b(x)
        return self._pw(self.proj2, self._pw(self.proj1, x, True), False)


def fno_block_flops(B: int, width: int, H: int, W: int, m1: int, m2: int) -> float:
    """Useful FLOPs of one FNO block (5 N log2 N per complex FFT-equivalent; real transforms
    counted at half; pointwise 2*C^2 per pixel; mixing 8*C^2 per kept mode)."""
    import math

    n = H * W
    fft = 2 * 0.5 * 5 * n * math.log2(n) * B * width
    mix = 8 * width * width * 2 * m1 * m2 * B
    pw = 2 * width * width * n * B
    return fft + mix + pw
