"""Operator layer: DFT ops (``dft``) and fused spectral-layer ops (``spectral``, ``nn``)."""
from .dft import (  # noqa: F401
    contrib_irfft, contrib_rfft, fft, fftn, ifft, ifftn, irfft, irfft2, irfftn, irfftn_pruned, norm_scale,
    rfft, rfft2, rfftn, rfftn_pruned,
)
