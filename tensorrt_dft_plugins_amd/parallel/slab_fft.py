"""Slab-decomposed distributed 2-D real FFT (the FFT analogue of sequence parallelism).

The reference is single-GPU only (/root/reference/src/dft_plugins/dft_plugins.cpp:341,
"assuming single GPU for now"; its batch is folded into the FFT, :249-266).  SURVEY §5.7 names
a slab decomposition as the way to go past one GPU's field size; this module implements it on
the hand-written kernels plus ONE collective per transform:

  rows local (R2C along W on this rank's H-slab)  ->  all_to_all transpose (RCCL over xGMI:
  every rank sends column block r to rank r -- each pair of GPUs talks over its own xGMI
  link, which is what a full-mesh 8-GPU node is good at)  ->  columns local (C2C along H on
  this rank's K-slab of the half spectrum).

Layouts (``P`` ranks, ``tensor_split``-balanced slabs, so any H and K work):
  rfft2 input : rank r holds rows  ``h_slab(H, P, r)`` of a real ``[..., H, W]`` field
  rfft2 output: rank r holds modes ``k_slab(W // 2 + 1, P, r)`` of the ``[..., H, W//2+1]``
                complex spectrum, all H frequencies
``slab_irfft2`` is the exact inverse (spectrum K-slabs in, real H-slabs out).  ``norm`` follows
torch.fft (``backward`` / ``ortho`` / ``forward``) over the full H x W transform.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..ops.dft import _ops, norm_scale


def _splits(n: int, p: int) -> List[int]:
    """Sizes of ``torch.tensor_split(range(n), p)``: the first n % p slabs are one larger."""
    q, r = divmod(n, p)
    return [q + (1 if i < r else 0) for i in range(p)]


def h_slab(H: int, world: int, rank: int) -> Tuple[int, int]:
    s = _splits(H, world)
    lo = sum(s[:rank])
    return lo, lo + s[rank]


def k_slab(K: int, world: int, rank: int) -> Tuple[int, int]:
    return h_slab(K, world, rank)


def _group_info(group) -> Tuple[int, int]:
    if group is None and not (dist.is_available() and dist.is_initialized()):
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def _all_to_all(send: List[torch.Tensor], recv_shapes: Sequence[Sequence[int]], group) -> List[torch.Tensor]:
    """One all_to_all_single over the concatenated flat blocks (uneven splits allowed)."""
    flat = torch.cat([b.reshape(-1) for b in send])
    in_splits = [b.numel() for b in send]
    out_splits = [int(torch.Size(s).numel()) for s in recv_shapes]
    out = torch.empty(sum(out_splits), dtype=flat.dtype, device=flat.device)
    dist.all_to_all_single(out, flat, out_splits, in_splits, group=group)
    return [c.reshape(s) for c, s in zip(out.split(out_splits), recv_shapes)]


def slab_rfft2(x_local: torch.Tensor, H: int, norm: Optional[str] = None, group=None) -> torch.Tensor:
    """Distributed ``rfft2`` over the last two dims of an H-slab-sharded real field.

    ``x_local``: ``[..., h_r, W]`` (this rank's rows ``h_slab(H, P, r)``).  Returns this rank's
    complex64 spectrum slab ``[..., H, k_r]`` (modes ``k_slab(W // 2 + 1, P, r)``).
    """
    rank, world = _group_info(group)
    W = x_local.shape[-1]
    K = W // 2 + 1
    lead = x_local.shape[:-2]
    hs = _splits(H, world)
    if x_local.shape[-2] != hs[rank]:
        raise ValueError(f"rank {rank}: expected {hs[rank]} rows of H={H}, got {x_local.shape[-2]}")
    # pass 1 (local): R2C along W, the whole transform's normalisation folded in here
    y = _ops().r2c(x_local.float().contiguous(), [x_local.dim() - 1], norm_scale(norm, H * W, True), [],
                   torch.float32)  # [..., h_r, K, 2]
    if world == 1:
        yt = y
    else:
        ks = _splits(K, world)
        bounds = [sum(ks[:i]) for i in range(world + 1)]
        send = [y[..., bounds[i]:bounds[i + 1], :].contiguous() for i in range(world)]
        recv = _all_to_all(send, [list(lead) + [hs[s], ks[rank], 2] for s in range(world)], group)
        yt = torch.cat(recv, dim=-3)  # [..., H, k_r, 2]
    # pass 2 (local): C2C along H on this rank's mode slab
    z = _ops().c2c(yt.contiguous(), [yt.dim() - 3], False, 1.0, torch.float32)
    return torch.view_as_complex(z)


def slab_irfft2(y_local: torch.Tensor, W: int, norm: Optional[str] = None, group=None) -> torch.Tensor:
    """Inverse of :func:`slab_rfft2`: ``y_local`` ``[..., H, k_r]`` complex (mode slab) ->
    this rank's real rows ``[..., h_r, W]`` (fp32)."""
    rank, world = _group_info(group)
    if not y_local.is_complex():
        raise TypeError("slab_irfft2 expects the complex spectrum slab")
    H = y_local.shape[-2]
    K = W // 2 + 1
    lead = y_local.shape[:-2]
    ks = _splits(K, world)
    if y_local.shape[-1] != ks[rank]:
        raise ValueError(f"rank {rank}: expected {ks[rank]} modes of K={K}, got {y_local.shape[-1]}")
    yr = torch.view_as_real(y_local.to(torch.complex64)).contiguous()  # [..., H, k_r, 2]
    # pass 1 (local): inverse C2C along H
    z = _ops().c2c(yr, [yr.dim() - 3], True, 1.0, torch.float32)
    hs = _splits(H, world)
    if world == 1:
        zt = z
    else:
        bounds = [sum(hs[:i]) for i in range(world + 1)]
        send = [z[..., bounds[i]:bounds[i + 1], :, :].contiguous() for i in range(world)]
        recv = _all_to_all(send, [list(lead) + [hs[rank], ks[s], 2] for s in range(world)], group)
        zt = torch.cat(recv, dim=-2)  # [..., h_r, K, 2]
    # pass 2 (local): C2R along W with the whole inverse normalisation
    return _ops().c2r(zt.contiguous(), [zt.dim() - 2], [W], norm_scale(norm, H * W, False), [], torch.float32)
