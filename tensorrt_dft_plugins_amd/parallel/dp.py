"""Batch data-parallel inference over RCCL (torch.distributed backend "nccl") / Gloo.

One process per GPU.  Each rank replays its own hipGraph-captured forward on
its batch shard; the per-step outputs are all-gathered over xGMI (RCCL
``all_gather_into_tensor``) on a dedicated communication stream, overlapped with the next
step's compute: two captured graphs write two output buffers (shared memory pool), and a
buffer is only overwritten after the collective that reads it has completed (stream-ordered
``work.wait()``, no host sync).  The reference has no parallelism at all
(/root/reference/src/dft_plugins/dft_plugins.cpp:341, "assuming single GPU").
"""
from __future__ import annotations

import os
from datetime import timedelta
from typing import List, Optional

import torch
import torch.distributed as dist

from ..engine.capture import CapturedModule


def init_distributed(backend: Optional[str] = None, timeout_s: float = 600.0) -> tuple[int, int, int]:
    """Initialise the default process group from torchrun env vars; returns (rank, world, local_rank).

    backend: "nccl" (= RCCL on ROCm) when a GPU is present, else "gloo"; ``MI_DFT_DIST_BACKEND``
    overrides (e.g. ``gloo`` to rehearse several ranks on ONE GPU, which RCCL refuses).
    """
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        if backend is None:
            backend = os.environ.get("MI_DFT_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, timeout=timedelta(seconds=timeout_s), device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend, timeout=timedelta(seconds=timeout_s))
    return rank, world, local


def world_info() -> tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def all_gather_batch(x: torch.Tensor, out: Optional[torch.Tensor] = None, async_op: bool = False,
                     force: bool = False):
    """Gather per-rank batch shards along dim 0 (RCCL all_gather_into_tensor; list form on Gloo).
    At world 1 this is a local copy unless ``force`` is set and a process group exists: then the
    collective itself runs (an RCCL communicator of one rank), so the comm path is exercised."""
    rank, world = world_info()
    if world == 1 and not (force and dist.is_available() and dist.is_initialized()):
        if out is not None:
            out.copy_(x)
            return out if not async_op else (out, None)
        return (x, None) if async_op else x
    if out is None:
        out = torch.empty((world * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    if dist.get_backend() == "gloo":
        parts = list(out.chunk(world, 0))
        w = dist.all_gather(parts, x.contiguous(), async_op=async_op)
    else:
        w = dist.all_gather_into_tensor(out, x.contiguous(), async_op=async_op)
    return (out, w) if async_op else out


def shard_checksum(t: torch.Tensor, chunk: int = 1 << 24) -> torch.Tensor:
    """Exact checksum of a tensor's bytes: (sum, position-weighted sum) of its 32/16/8-bit words as
    int64 (wrap-around arithmetic), so any changed, missing or permuted word shows up.  Computed in
    chunks (no full-size int64 copy).  Returns a [2] int64 tensor on the CPU."""
    flat = t.contiguous().view(-1)
    nbytes = flat.numel() * flat.element_size()
    wt = torch.int32 if nbytes % 4 == 0 else (torch.int16 if nbytes % 2 == 0 else torch.uint8)
    words = flat.view(torch.uint8).view(wt)
    s0 = torch.zeros((), dtype=torch.int64, device=t.device)
    s1 = torch.zeros((), dtype=torch.int64, device=t.device)
    for a in range(0, words.numel(), chunk):
        w = words[a:a + chunk].to(torch.int64)
        idx = torch.arange(a, a + w.numel(), dtype=torch.int64, device=t.device) % 65521 + 1
        s0 += w.sum()
        s1 += (w * idx).sum()
    return torch.stack([s0, s1]).cpu()


_HOST_GROUP = {}


def _host_group():
    """A Gloo group over the default group's ranks for host-side exchanges (created once per default
    process group: ``new_group`` is collective, so every rank reaches this in the same order)."""
    if dist.get_backend() == "gloo":
        return None
    world = dist.group.WORLD
    # keyed by the group object itself (held here, so a later default group cannot reuse its id)
    if _HOST_GROUP.get("world") is not world:
        _HOST_GROUP["world"] = world
        _HOST_GROUP["gloo"] = dist.new_group(backend="gloo")
    return _HOST_GROUP["gloo"]


def ipc_peer_access_problem(device: torch.device) -> Optional[str]:
    """Why the direct IPC mesh cannot span the ranks (None if it can): every rank's device index is
    all-gathered and each rank checks ``hipDeviceCanAccessPeer`` to every peer's device; one
    failing pair anywhere makes every rank fall back (the verdict is all-reduced)."""
    from .._loader import load_plugins

    rank, world = world_info()
    dev = device.index if device.index is not None else torch.cuda.current_device()
    devs: List[Optional[int]] = [None] * world
    grp = None
    if world > 1:
        grp = _host_group()
        dist.all_gather_object(devs, dev, group=grp)
    else:
        devs = [dev]
    load_plugins()
    bad = []
    for p, d in enumerate(devs):
        if p == rank:
            continue
        if d == dev:
            continue  # several ranks on one GPU (Gloo rehearsal): same-device IPC needs no peer link
        if not torch.ops.amd_dft._ipc_can_access_peer(dev, int(d)):
            bad.append((rank, p, dev, int(d)))
    n = torch.tensor([len(bad)], dtype=torch.int64)
    if world > 1:
        dist.all_reduce(n, group=grp)
    if int(n.item()) == 0:
        return None
    mine = f" (rank {rank}: no peer access to {[(p, d) for _, p, _, d in bad]})" if bad else ""
    return f"hipDeviceCanAccessPeer false for {int(n.item())} rank pair(s){mine}"


class DataParallelInference:
    """Overlapped batch-DP inference of a static-shape module (per-rank shard = ``example``).

    ``gather_backend``: ``"rccl"`` (``all_gather_into_tensor``; Gloo on CPU) or ``"ipc"`` (direct
    pushes into every peer's buffer over xGMI, :mod:`.ipc_gather`); default from
    ``MI_DFT_GATHER``, else rccl.
    ``gather_dtype``: e.g. ``torch.bfloat16`` gathers a reduced-precision copy of the output
    (SURVEY §5.8 plan item 3: half the xGMI bytes of an fp32 model's output); the cast is part
    of the captured graph, and the gathered buffers have that dtype.  Default: the output dtype.
    ``force_gather``: run the gather (and its comm-stream ordering) even at world 1, provided a
    process group exists -- an RCCL communicator of one rank on one GPU executes the same
    ``all_gather_into_tensor`` / stream-ordered ``work.wait()`` path an 8-GPU job runs.
    With ``gather_backend="ipc"`` the direct mesh is only built when every pair of ranks reports
    peer access (``hipDeviceCanAccessPeer``); otherwise the runner falls back to RCCL and records
    why in ``gather_fallback``.
    """

    def __init__(self, module, example: torch.Tensor, *, gather: bool = True,
                 use_graph: bool = True, warmup: int = 2, gather_backend: Optional[str] = None,
                 gather_dtype: Optional[torch.dtype] = None, force_gather: bool = False):
        self.rank, self.world = world_info()
        self.force_gather = bool(force_gather) and dist.is_available() and dist.is_initialized()
        self.gather = gather and (self.world > 1 or self.force_gather)
        self.gather_backend = (gather_backend or os.environ.get("MI_DFT_GATHER", "rccl")).lower()
        if self.gather_backend not in ("rccl", "ipc"):
            raise ValueError(f"gather_backend must be 'rccl' or 'ipc', got {self.gather_backend!r}")
        self.gather_fallback: Optional[str] = None
        if self.gather and self.gather_backend == "ipc" and example.device.type == "cuda":
            why = ipc_peer_access_problem(example.device)
            if why is not None:
                self.gather_fallback = f"ipc -> rccl: {why}"
                self.gather_backend = "rccl"
        self.gather_dtype = gather_dtype if self.gather else None
        fn = module
        if self.gather_dtype is not None:
            gd = self.gather_dtype

            def fn(*xs):  # noqa: F811  (cast captured with the forward)
                o = module(*xs)
                return o.to(gd) if o.dtype != gd else o
        self.cap = CapturedModule(fn, [example], warmup=warmup, n_graphs=2 if self.gather else 1,
                                  use_graph=use_graph)
        self.device = example.device
        self.cuda = self.device.type == "cuda"
        self.comm_stream = torch.cuda.Stream(self.device) if self.cuda else None
        self.full: List[Optional[torch.Tensor]] = [None, None]
        self.works: List[Optional[object]] = [None, None]
        self.events = [torch.cuda.Event() if self.cuda else None for _ in range(2)]
        self.done = [torch.cuda.Event() if self.cuda else None for _ in range(2)]
        self.done_pending = [False, False]
        self.ipc = None
        if self.gather:
            o = self.cap.outputs[0][0]
            if self.gather_backend == "ipc":
                from .ipc_gather import IpcAllGather

                self.ipc = IpcAllGather(list(o.shape), o.dtype, o.device, nbuf=2)
                self.full = list(self.ipc.full)
            else:
                for i in range(2):
                    self.full[i] = torch.empty((self.world * o.shape[0],) + tuple(o.shape[1:]), dtype=o.dtype,
                                               device=o.device)
        self.k = 0
        self._comm_marks: Optional[List[tuple]] = None  # (start, end) events per gather when timing

    # ------------------------------------------------------------------ diagnostics
    def time_comm(self, on: bool = True) -> None:
        """Record a (start, end) event pair around every gather on the comm stream (GPU)."""
        self._comm_marks = [] if on and self.cuda and self.gather else None

    def comm_busy_ms(self) -> Optional[float]:
        """Total comm-stream time spent inside gathers since ``time_comm()`` (call after ``drain``
        + synchronize).  The start event sits after the wait for the step's compute, so this is
        the gathers' own duration, not their queueing behind compute."""
        if self._comm_marks is None:
            return None
        return float(sum(a.elapsed_time(b) for a, b in self._comm_marks))

    def gather_only_ms(self, iters: int = 5) -> Optional[float]:
        """Milliseconds per gather with no compute in flight: ``iters`` back-to-back gathers of
        the current output shard (the xGMI / RCCL cost the overlapped step hides)."""
        if not self.gather:
            return None
        self.drain()
        out = self.cap.outputs[0][0]
        if self.cuda:
            torch.cuda.synchronize(self.device)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(self.comm_stream):
                self.comm_stream.wait_stream(torch.cuda.current_stream(self.device))
                a.record(self.comm_stream)
                for j in range(iters):
                    if self.ipc is not None:
                        self.ipc.gather(out, j)
                    else:
                        all_gather_batch(out, self.full[0], async_op=False, force=self.force_gather)
                b.record(self.comm_stream)
            torch.cuda.synchronize(self.device)
            return a.elapsed_time(b) / iters
        import time as _t

        t0 = _t.perf_counter()
        for j in range(iters):
            if self.ipc is not None:
                self.ipc.gather(out, j)
            else:
                all_gather_batch(out, self.full[0], async_op=False, force=self.force_gather)
        if self.ipc is not None:
            self.ipc.synchronize()
        return (_t.perf_counter() - t0) * 1e3 / iters

    @property
    def inputs(self) -> torch.Tensor:
        return self.cap.inputs[0]

    def step(self) -> torch.Tensor:
        """Enqueue one step; returns the gathered output buffer of this step.

        The buffer is complete only in stream order: read it after ``drain()`` (GPU: the current
        stream then waits for the gather; CPU: the gather has finished) -- on the CPU/IPC path the
        pushes run asynchronously on a worker thread, exactly as on the GPU.  It stays valid until
        the step two calls later reuses its slot."""
        i = self.k % len(self.cap.outputs)
        self.k += 1
        if self.gather and self.works[i] is not None:
            self.works[i].wait()  # stream-ordered: compute waits until the old gather read out[i]
            self.works[i] = None
        if self.cuda and self.done_pending[i]:
            torch.cuda.current_stream(self.device).wait_event(self.done[i])  # old push has read out[i]
            self.done_pending[i] = False
        out = self.cap.replay(i)[0]
        if not self.gather:
            return out
        marks = None
        if self._comm_marks is not None:
            marks = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            self._comm_marks.append(marks)
        if self.ipc is not None:
            if self.cuda:
                self.events[i].record()
                with torch.cuda.stream(self.comm_stream):
                    self.comm_stream.wait_event(self.events[i])
                    if marks:
                        marks[0].record(self.comm_stream)
                    self.ipc.gather(out, i)
                    if marks:
                        marks[1].record(self.comm_stream)
                    self.done[i].record(self.comm_stream)
                self.done_pending[i] = True
            else:
                self.ipc.gather(out, i)
            return self.full[i]
        if self.cuda:
            self.events[i].record()
            with torch.cuda.stream(self.comm_stream):
                self.comm_stream.wait_event(self.events[i])
                if marks:
                    marks[0].record(self.comm_stream)
                _, self.works[i] = all_gather_batch(out, self.full[i], async_op=True, force=self.force_gather)
                if marks:
                    # RCCL runs on its own stream: join it (stream-ordered, no host wait) so the
                    # end mark is recorded when the collective has finished
                    self.works[i].wait()
                    marks[1].record(self.comm_stream)
        else:
            _, self.works[i] = all_gather_batch(out, self.full[i], async_op=True, force=self.force_gather)
        return self.full[i]

    def last_slot(self) -> Optional[int]:
        """Buffer slot written by the most recent ``step()`` (None before the first)."""
        return None if self.k == 0 else (self.k - 1) % len(self.cap.outputs)

    def verify_gather(self) -> dict:
        """Collective self-check of the last step's gather: rank r's slot of the gathered buffer
        must be bit-identical to rank r's local output.  Every rank computes exact integer
        checksums (:func:`shard_checksum`) of its local output and of every slot of its gathered
        buffer; the local ones are all-gathered, and each rank compares slot r against rank r's
        local checksum.  Returns ``{"gather_verified": bool, "gather_mismatches": n}`` (the
        mismatch count summed over ranks, so every rank returns the same verdict)."""
        if not self.gather or self.k == 0:
            return {"gather_verified": None, "gather_mismatches": 0}
        self.drain()
        if self.cuda:
            torch.cuda.synchronize(self.device)
        i = self.last_slot()
        local = self.cap.outputs[i][0]
        full = self.full[i]
        mine = shard_checksum(local)
        slots = torch.stack([shard_checksum(c) for c in full.chunk(self.world, 0)])  # [world, 2]
        dev = self.device if (self.cuda and dist.get_backend() != "gloo") else torch.device("cpu")
        if self.world > 1 or self.force_gather:
            everyone = torch.empty(self.world, 2, dtype=torch.int64, device=dev)
            all_gather_batch(mine.view(1, 2).to(dev), everyone, force=self.force_gather)
        else:
            everyone = mine.view(1, 2)
        bad = int((everyone.cpu() != slots.cpu()).any(dim=1).sum())
        tot = torch.tensor([bad], dtype=torch.int64, device=dev)
        if self.world > 1:
            dist.all_reduce(tot)
        n = int(tot.item())
        return {"gather_verified": n == 0, "gather_mismatches": n}

    def drain(self) -> None:
        """Make the current stream wait for all outstanding gathers (CPU: until they are done)."""
        for i, w in enumerate(self.works):
            if w is not None:
                w.wait()
                self.works[i] = None
        if self.cuda:
            torch.cuda.current_stream(self.device).wait_stream(self.comm_stream)
        elif self.ipc is not None:
            self.ipc.synchronize()

    def close(self) -> None:
        """Collective teardown: finish every gather, then (IPC) barrier and release the peer
        handles before the gather buffers are freed (no peer may still push into them)."""
        self.drain()
        if self.cuda:
            torch.cuda.synchronize(self.device)
        if self.ipc is not None:
            self.ipc.close()
            self.ipc = None
        self.full = [None, None]

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False
