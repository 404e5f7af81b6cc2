"""Functional DFT API on top of the native ``torch.ops.amd_dft`` kernels.

* ``contrib_rfft`` / ``contrib_irfft``: the ONNX-Runtime contrib ``Rfft``/``Irfft``
  semantics implemented by the reference plugins (real tensors with a trailing re/im dim of
  size 2, "backward" normalisation, last ``signal_ndim`` dims;
  /root/reference/src/dft_plugins/dft_plugins.cpp:361-382, :415-436, :457-468).
* ``rfft``/``irfft``/``rfft2``/``irfft2``/``rfftn``/``irfftn``/``fft``/``ifft``/``fftn``/``ifftn``:
  ``torch.fft``-compatible signatures (any dims, including channel-last layouts such as the
  AFNO ``dim=(1, 2)`` case), backed by the hand-written Stockham kernels on MI355X.
* ``rfftn_pruned`` / ``irfftn_pruned``: mode-truncated transforms used by the FNO/AFNO
  spectral layers (only the kept modes are ever computed / stored).

bf16 inputs are supported with fp32 internal compute (``torch.fft`` rejects bf16).
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import torch

from .._loader import load_plugins

__all__ = [
    "contrib_rfft", "contrib_irfft", "rfft", "irfft", "rfft2", "irfft2", "rfftn", "irfftn",
    "fft", "ifft", "fftn", "ifftn", "rfftn_pruned", "irfftn_pruned", "norm_scale",
]


def _ops():
    load_plugins()
    return torch.ops.amd_dft


def norm_scale(norm: Optional[str], n: int, forward: bool) -> float:
    norm = norm or "backward"
    if norm == "backward":
        return 1.0 if forward else 1.0 / n
    if norm == "ortho":
        return 1.0 / math.sqrt(n)
    if norm == "forward":
        return 1.0 / n if forward else 1.0
    raise ValueError(f"invalid norm {norm!r}")


def _as_list(dim) -> list[int]:
    if isinstance(dim, int):
        return [dim]
    return list(dim)


def _resize(x: torch.Tensor, dim: int, n: int) -> torch.Tensor:
    """Zero-pad or trim ``x`` along ``dim`` to length ``n`` (torch.fft ``n=`` semantics)."""
    cur = x.shape[dim]
    if n == cur:
        return x
    if n < cur:
        return x.narrow(dim, 0, n)
    pad_shape = list(x.shape)
    pad_shape[dim] = n - cur
    return torch.cat([x, x.new_zeros(pad_shape)], dim=dim)


def _to_complex(y: torch.Tensor) -> torch.Tensor:
    if y.dtype == torch.float32:
        return torch.view_as_complex(y)
    return torch.view_as_complex(y.float().contiguous())


def _from_complex(x: torch.Tensor) -> torch.Tensor:
    if x.is_complex():
        return torch.view_as_real(x.to(torch.complex64).resolve_conj())
    if x.shape[-1] != 2:
        raise ValueError("expected a complex tensor or a real tensor with a trailing dim of size 2")
    return x


# ----------------------------------------------------------------- ONNX-contrib parity
def contrib_rfft(x: torch.Tensor, signal_ndim: int = 1, normalized: int = 0, onesided: int = 1) -> torch.Tensor:
    """``com.microsoft::Rfft``: real ``[..., n1..ns]`` -> ``[..., n1.., ns//2+1, 2]``."""
    return _ops().Rfft(x, normalized, onesided, signal_ndim)


def contrib_irfft(x: torch.Tensor, signal_ndim: int = 1, normalized: int = 0, onesided: int = 1) -> torch.Tensor:
    """``com.microsoft::Irfft``: ``[..., m, 2]`` -> real ``[..., 2(m-1)]`` scaled by 1/N."""
    return _ops().Irfft(x, normalized, onesided, signal_ndim)


# ----------------------------------------------------------------- torch.fft-like API
def rfftn(x: torch.Tensor, s: Optional[Sequence[int]] = None, dim: Optional[Sequence[int]] = None,
          norm: Optional[str] = None, *, return_real: bool = False,
          out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    if x.is_complex():
        raise TypeError("rfftn expects a real input")
    if dim is None:
        dim = list(range(x.dim() - len(s), x.dim())) if s is not None else list(range(x.dim()))
    dim = [d % x.dim() for d in _as_list(dim)]
    if s is not None:
        for d, n in zip(dim, s):
            x = _resize(x, d, n)
    n_total = 1
    for d in dim:
        n_total *= x.shape[d]
    y = _ops().r2c(x, dim, norm_scale(norm, n_total, True), [], out_dtype or (x.dtype if return_real else torch.float32))
    return y if return_real else _to_complex(y)


def irfftn(x: torch.Tensor, s: Optional[Sequence[int]] = None, dim: Optional[Sequence[int]] = None,
           norm: Optional[str] = None, *, out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    xr = _from_complex(x)
    nd = xr.dim() - 1
    if dim is None:
        dim = list(range(nd - len(s), nd)) if s is not None else list(range(nd))
    dim = [d % nd for d in _as_list(dim)]
    order = sorted(range(len(dim)), key=lambda i: dim[i])
    dim_sorted = [dim[i] for i in order]
    if s is None:
        sizes = [xr.shape[d] for d in dim_sorted]
        sizes[-1] = 2 * (sizes[-1] - 1)
    else:
        s = list(s)
        sizes = [s[i] for i in order]
    for d, n in zip(dim_sorted[:-1], sizes[:-1]):
        xr = _resize(xr, d, n)
    # last dim: stored count may exceed n//2+1 (truncated) or be shorter (zero modes)
    n_total = 1
    for n in sizes:
        n_total *= n
    odt = out_dtype or (torch.float32 if x.is_complex() else xr.dtype)
    return _ops().c2r(xr, dim_sorted, sizes, norm_scale(norm, n_total, False), [], odt)


def rfft(x, n: Optional[int] = None, dim: int = -1, norm: Optional[str] = None, **kw):
    return rfftn(x, None if n is None else [n], [dim], norm, **kw)


def irfft(x, n: Optional[int] = None, dim: int = -1, norm: Optional[str] = None, **kw):
    return irfftn(x, None if n is None else [n], [dim], norm, **kw)


def rfft2(x, s=None, dim=(-2, -1), norm: Optional[str] = None, **kw):
    return rfftn(x, s, dim, norm, **kw)


def irfft2(x, s=None, dim=(-2, -1), norm: Optional[str] = None, **kw):
    return irfftn(x, s, dim, norm, **kw)


def fftn(x: torch.Tensor, s=None, dim=None, norm: Optional[str] = None, *, inverse: bool = False,
         return_real: bool = False) -> torch.Tensor:
    """C2C transform; a real input is promoted to complex (imaginary part zero)."""
    if x.is_complex():
        xr = _from_complex(x)
    else:
        xr = torch.stack([x.float(), torch.zeros_like(x, dtype=torch.float32)], dim=-1)
    nd = xr.dim() - 1
    if dim is None:
        dim = list(range(nd - len(s), nd)) if s is not None else list(range(nd))
    dim = [d % nd for d in _as_list(dim)]
    if s is not None:
        for d, n in zip(dim, s):
            xr = _resize(xr, d, n)
    n_total = 1
    for d in dim:
        n_total *= xr.shape[d]
    y = _ops().c2c(xr, dim, inverse, norm_scale(norm, n_total, not inverse), torch.float32)
    return y if return_real else _to_complex(y)


def ifftn(x, s=None, dim=None, norm: Optional[str] = None, **kw):
    return fftn(x, s, dim, norm, inverse=True, **kw)


def fft(x, n: Optional[int] = None, dim: int = -1, norm: Optional[str] = None, **kw):
    return fftn(x, None if n is None else [n], [dim], norm, **kw)


def ifft(x, n: Optional[int] = None, dim: int = -1, norm: Optional[str] = None, **kw):
    return fftn(x, None if n is None else [n], [dim], norm, inverse=True, **kw)


# ----------------------------------------------------------------- pruned (mode-truncated)
def rfftn_pruned(x: torch.Tensor, dim: Sequence[int], keep: Sequence[tuple[int, int]], norm: Optional[str] = None,
                 out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """R2C keeping only modes ``[0, lo) u [n-hi, n)`` per dim (innermost dim: ``[0, lo)``).

    Returns a real tensor with a trailing re/im dim.  Dims are given in any order; ``keep``
    follows ``dim``.
    """
    dim = [d % x.dim() for d in dim]
    n_total = 1
    for d in dim:
        n_total *= x.shape[d]
    flat = [v for kv in keep for v in kv]
    return _ops().r2c(x, dim, norm_scale(norm, n_total, True), flat, out_dtype or torch.float32)


def irfftn_pruned(x: torch.Tensor, dim: Sequence[int], out_size: Sequence[int], keep: Sequence[tuple[int, int]],
                  norm: Optional[str] = None, out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """Inverse of :func:`rfftn_pruned`: ``x`` stores only the kept modes (zeros elsewhere)."""
    nd = x.dim() - 1
    dim = [d % nd for d in dim]
    n_total = 1
    for n in out_size:
        n_total *= n
    flat = [v for kv in keep for v in kv]
    return _ops().c2r(x, dim, list(out_size), norm_scale(norm, n_total, False), flat, out_dtype or torch.float32)
