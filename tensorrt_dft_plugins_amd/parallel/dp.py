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


def all_gather_batch(x: torch.Tensor, out: Optional[torch.Tensor] = None, async_op: bool = False):
    """Gather per-rank batch shards along dim 0 (RCCL all_gather_into_tensor; list form on Gloo)."""
    rank, world = world_info()
    if world == 1:
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


class DataParallelInference:
    """Overlapped batch-DP inference of a static-shape module (per-rank shard = ``example``).

    ``gather_backend``: ``"rccl"`` (``all_gather_into_tensor``; Gloo on CPU) or ``"ipc"`` (direct
    pushes into every peer's buffer over xGMI, :mod:`.ipc_gather`); default from
    ``MI_DFT_GATHER``, else rccl.
    ``gather_dtype``: e.g. ``torch.bfloat16`` gathers a reduced-precision copy of the output
    (SURVEY §5.8 plan item 3: half the xGMI bytes of an fp32 model's output); the cast is part
    of the captured graph, and the gathered buffers have that dtype.  Default: the output dtype.
    """

    def __init__(self, module, example: torch.Tensor, *, gather: bool = True,
                 use_graph: bool = True, warmup: int = 2, gather_backend: Optional[str] = None,
                 gather_dtype: Optional[torch.dtype] = None):
        self.rank, self.world = world_info()
        self.gather = gather and self.world > 1
        self.gather_backend = (gather_backend or os.environ.get("MI_DFT_GATHER", "rccl")).lower()
        if self.gather_backend not in ("rccl", "ipc"):
            raise ValueError(f"gather_backend must be 'rccl' or 'ipc', got {self.gather_backend!r}")
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
                        all_gather_batch(out, self.full[0], async_op=False)
                b.record(self.comm_stream)
            torch.cuda.synchronize(self.device)
            return a.elapsed_time(b) / iters
        import time as _t

        t0 = _t.perf_counter()
        for j in range(iters):
            if self.ipc is not None:
                self.ipc.gather(out, j)
            else:
                all_gather_batch(out, self.full[0], async_op=False)
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
                _, self.works[i] = all_gather_batch(out, self.full[i], async_op=True)
                if marks:
                    # RCCL runs on its own stream: join it (stream-ordered, no host wait) so the
                    # end mark is recorded when the collective has finished
                    self.works[i].wait()
                    marks[1].record(self.comm_stream)
        else:
            _, self.works[i] = all_gather_batch(out, self.full[i], async_op=True)
        return self.full[i]

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
