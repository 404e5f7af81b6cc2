"""Direct-mesh all-gather of the batch-DP output over xGMI (the C-1 call site).

RCCL's ring all-gather moves every shard through ``world - 1`` hops, so at 8 GPUs a rank's
links carry 7 shards each way in sequence; the MI355X's xGMI is a full point-to-point mesh, so
each rank can instead PUSH its shard straight into every peer's output buffer -- ``world - 1``
concurrent copies, one per link, each moving one shard (ring: ~7 x shard / link bandwidth;
mesh: ~1 x shard / link bandwidth, derived in SURVEY §5.8).

Protocol per step (buffer slot ``i`` of ``nbuf``, all on the caller's current stream):
  1. push: one kernel (csrc/parallel/ipc_push.hip) stores the local shard into slot ``i`` of every
     rank's buffer at once (peer pointers from ``hipIpcOpenMemHandle``; one xGMI link per peer),
     at byte offset ``rank * shard_bytes``;
  2. record this rank's inter-process event ``i`` after the pushes;
  3. host handshake: a barrier on a Gloo group -- afterwards every producer has ENQUEUED its
     pushes and its event record for this step (the host never waits for the GPU);
  4. the stream waits on every peer's event ``i``: stream-ordered completion of all pushes.
A slot is rewritten ``nbuf`` steps later, so the gathered buffer of a step stays valid while
the next ``nbuf - 1`` steps are enqueued (the DP runner's double-buffer contract).

Transports: ``HipIpcTransport`` (GPU: hipMalloc'd buffers, IPC memory/event handles) and
``ShmTransport`` (CPU: ``/dev/shm``-backed storages, synchronous copies) -- the latter runs the
same slot / offset / handshake logic in multi-process Gloo tests without a GPU.
"""
from __future__ import annotations

import os
import uuid
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from .._loader import load_plugins


class HipIpcTransport:
    """hipMalloc'd gather buffers shared through IPC memory / event handles."""

    def __init__(self, device: torch.device):
        load_plugins()
        self.device = device
        self.dev = device.index if device.index is not None else torch.cuda.current_device()
        self.ops = torch.ops.amd_dft
        self._opened: List[int] = []
        self._events: List[int] = []

    def alloc(self, nbytes: int):
        buf = self.ops._ipc_alloc(nbytes, self.dev)
        return buf, self.ops._ipc_mem_handle(buf)

    def open(self, handle, local_buf, is_self: bool) -> int:
        if is_self:  # a process cannot open its own handle: use the buffer directly
            return local_buf.data_ptr()
        p = self.ops._ipc_open_mem(handle, self.dev)
        self._opened.append(p)
        return p

    def new_event(self):
        ev = self.ops._ipc_event_create(self.dev)
        self._events.append(ev)
        return ev, self.ops._ipc_event_handle(ev)

    def open_event(self, handle, local_ev, is_self: bool):
        return local_ev if is_self else self.ops._ipc_event_open(handle, self.dev)

    def push(self, src: torch.Tensor, dst_ptrs: Sequence[int], offset: int) -> None:
        self.ops._ipc_push(src.contiguous(), list(dst_ptrs), offset)

    def record(self, ev) -> None:
        self.ops._ipc_event_record(ev, self.dev)

    def wait(self, ev) -> None:
        self.ops._ipc_stream_wait(ev, self.dev)

    def close(self) -> None:
        for p in self._opened:
            self.ops._ipc_close_mem(p)
        for ev in self._events:
            self.ops._ipc_event_destroy(ev)
        self._opened, self._events = [], []


class ShmTransport:
    """CPU stand-in: each buffer is a ``/dev/shm`` file mapped by every rank; copies are
    synchronous, events are no-ops (the host handshake already orders them)."""

    def __init__(self, device: torch.device = torch.device("cpu")):
        self.device = device
        self._files: List[str] = []

    def alloc(self, nbytes: int):
        path = f"/dev/shm/amd_dft_ipc_{os.getpid()}_{uuid.uuid4().hex[:12]}"
        st = torch.UntypedStorage.from_file(path, shared=True, nbytes=nbytes)
        self._files.append(path)
        return torch.empty(0, dtype=torch.uint8).set_(st), (path, nbytes)

    def open(self, handle, local_buf, is_self: bool):
        if is_self:
            return local_buf
        path, nbytes = handle
        return torch.empty(0, dtype=torch.uint8).set_(torch.UntypedStorage.from_file(path, shared=True, nbytes=nbytes))

    def new_event(self):
        return None, None

    def open_event(self, handle, local_ev, is_self: bool):
        return None

    def push(self, src: torch.Tensor, dsts, offset: int) -> None:
        b = src.contiguous().view(torch.uint8).reshape(-1)
        for d in dsts:
            d[offset:offset + b.numel()].copy_(b)

    def record(self, ev) -> None:
        pass

    def wait(self, ev) -> None:
        pass

    def close(self) -> None:
        for f in self._files:
            try:
                os.unlink(f)
            except OSError:
                pass
        self._files = []


class IpcAllGather:
    """All-gather of a fixed-shape shard along dim 0 by direct pushes (see module docstring).

    ``gather(local, i)`` returns slot ``i``'s ``[world * shard_shape[0], ...]`` tensor, complete
    in stream order.  Collective: every rank constructs it with the same arguments.
    """

    def __init__(self, shard_shape: Sequence[int], dtype: torch.dtype, device: torch.device, *, nbuf: int = 2,
                 transport=None, group=None):
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.shard_shape = list(shard_shape)
        self.dtype = dtype
        self.nbuf = nbuf
        self.device = device
        self.transport = transport or (HipIpcTransport(device) if device.type == "cuda" else ShmTransport())
        # host-side handshake group: Gloo never waits for the GPU
        self.host_group = group if group is not None else (
            dist.new_group(backend="gloo") if dist.get_backend() != "gloo" else dist.group.WORLD)
        elem = torch.empty(0, dtype=dtype).element_size()
        self.shard_bytes = int(torch.Size(self.shard_shape).numel()) * elem
        full_shape = [self.world * self.shard_shape[0]] + self.shard_shape[1:]
        self.full: List[torch.Tensor] = []
        self.peers: List[List[object]] = []
        self.events: List[object] = []
        self.peer_events: List[List[object]] = []
        for _ in range(nbuf):
            buf, handle = self.transport.alloc(self.world * self.shard_bytes)
            ev, ev_handle = self.transport.new_event()
            handles: List[Optional[object]] = [None] * self.world
            dist.all_gather_object(handles, (handle, ev_handle), group=self.host_group)
            self.full.append(buf.view(dtype).view(full_shape))
            self.peers.append([self.transport.open(h[0], buf, p == self.rank) for p, h in enumerate(handles)])
            self.events.append(ev)
            self.peer_events.append([self.transport.open_event(h[1], ev, p == self.rank) for p, h in enumerate(handles)])
        dist.barrier(group=self.host_group)

    def gather(self, local: torch.Tensor, i: int) -> torch.Tensor:
        if list(local.shape) != self.shard_shape or local.dtype != self.dtype:
            raise ValueError(f"shard {list(local.shape)} {local.dtype} != {self.shard_shape} {self.dtype}")
        i %= self.nbuf
        self.transport.push(local, self.peers[i], self.rank * self.shard_bytes)
        self.transport.record(self.events[i])
        dist.barrier(group=self.host_group)
        for p in range(self.world):
            if p != self.rank:
                self.transport.wait(self.peer_events[i][p])
        return self.full[i]

    def close(self) -> None:
        dist.barrier(group=self.host_group)
        self.transport.close()
