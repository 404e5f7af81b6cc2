"""Direct-mesh all-gather of the batch-DP output over xGMI (the C-1 call site).

RCCL's ring all-gather moves every shard through ``world - 1`` hops, so at 8 GPUs a rank's
links carry 7 shards each way in sequence; the MI355X's xGMI is a full point-to-point mesh, so
each rank can instead PUSH its shard straight into every peer's output buffer -- ``world - 1``
concurrent copies, one per link, each moving one shard (ring: ~7 x shard / link bandwidth;
mesh: ~1 x shard / link bandwidth, derived in SURVEY §5.8).

Protocol per step, ``protocol="flags"`` (opt-in; buffer slot ``i`` of ``nbuf``, its ``n``-th use,
all on the caller's current stream, no host handshake):
  1. release: write ``n`` into flag word (slot i, REL, this rank) of every PEER's flag buffer
     (``hipStreamWriteValue32``, stream-ordered after everything this rank enqueued before the
     call -- in particular every consumer of the slot's previous contents);
  2. the stream waits until this rank's own flag words (i, REL, p) >= n for every peer p
     (``hipStreamWaitValue32``): a push never overwrites a peer's slot while that peer's GPU may
     still read the old contents (write-after-read across processes);
  3. push: one kernel (csrc/parallel/ipc_push.hip) stores the local shard into slot ``i`` of every
     rank's buffer at once (peer pointers from ``hipIpcOpenMemHandle``; one xGMI link per peer),
     at byte offset ``rank * shard_bytes``;
  4. write ``n`` into (i, DONE, this rank) of every peer's flags after the pushes;
  5. the stream waits until its own (i, DONE, p) >= n for every peer: all pushes into this rank's
     slot have completed.
A wait on a counter value (not on "the latest record" of an event) is satisfied by exactly the
peer's n-th release / push whenever the peer gets to it, so no rank has to know that the others
have enqueued their records: the gather enqueues 4 (world - 1) stream packets and returns, and the
host never blocks on a peer (no barriers on the enqueue path).
``protocol="events"`` (default) is the round-2 form: inter-process events, whose stream wait
targets the latest record enqueued so far, so two Gloo host barriers per step ensure the peers'
records are enqueued first.  It stays the default until the flag protocol has been validated
across xGMI (gathered contents checked over slot reuse on a multi-GPU node): the event record /
wait pair is a system-scope release / acquire that the runtime provides, whereas the flag words
rely on the push kernel's own system-scope release (csrc/parallel/ipc_push.hip).
Failure behaviour: with "events" a dead peer surfaces as a Gloo barrier timeout (the process
group's timeout, ``init_distributed(timeout_s=...)``); with "flags" the host never blocks, so a
dead peer leaves this rank's STREAM waiting on a flag word that never advances -- the next host
synchronisation (``drain()`` + ``torch.cuda.synchronize``) hangs.  Bound it from outside (job-level
timeout), or use "events" where a peer may die.
Contract (both): the gathered buffer of step ``k`` stays valid until the gather of step
``k + nbuf`` is called, and every read of it must be enqueued (in stream order on the calling
stream, or joined into it) before that call.

Transports: ``HipIpcTransport`` (GPU: hipMalloc'd buffers, IPC memory/event handles) and
``ShmTransport`` (CPU: ``/dev/shm``-backed storages).  The CPU transport emulates a GPU stream
with one worker thread per rank, inter-process events with shared ``(enqueued, completed)``
counters and flag words as shared int32s written / polled by the workers, so the multi-process
Gloo tests exercise the same ordering the GPU relies on -- a deliberately slow consumer on one
rank shows whether a peer's push waits for it (tests/test_dp.py::test_ipc_gather_slow_consumer_*).
"""
from __future__ import annotations

import os
import queue
import threading
import time
import uuid
from typing import Callable, List, Optional, Sequence

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
        self._opened: List[int] = []         # peers' buffers mapped into this process
        self._opened_events: List[int] = []  # peers' events opened in this process
        self._events: List[int] = []         # this rank's own (exported) events
        self._bufs: List[torch.Tensor] = []  # this rank's own (exported) buffers

    def alloc(self, nbytes: int):
        buf = self.ops._ipc_alloc(nbytes, self.dev)
        self._bufs.append(buf)
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
        if is_self:
            return local_ev
        ev = self.ops._ipc_event_open(handle, self.dev)
        self._opened_events.append(ev)
        return ev

    def push(self, src: torch.Tensor, dst_ptrs: Sequence[int], offset: int) -> None:
        self.ops._ipc_push(src.contiguous(), list(dst_ptrs), offset)

    def record(self, ev) -> None:
        self.ops._ipc_event_record(ev, self.dev)

    def wait(self, ev) -> None:
        self.ops._ipc_stream_wait(ev, self.dev)

    def write_value(self, flags, idx: int, value: int) -> None:
        self.ops._ipc_write_value(int(flags) + 4 * idx, value, self.dev)

    def wait_value(self, flags, idx: int, value: int) -> None:
        self.ops._ipc_wait_value(int(flags) + 4 * idx, value, self.dev)

    def enqueue(self, fn: Callable[[], None]) -> None:
        fn()  # device work is already stream-ordered: run the enqueueing code now

    def synchronize(self) -> None:
        torch.cuda.current_stream(self.device).synchronize()

    def close_imports(self) -> None:
        """Teardown step 1: unmap every peer buffer and release every peer event this process
        opened.  Caller guarantees (barrier) that no rank still pushes or waits."""
        torch.cuda.synchronize(self.device)
        for p in self._opened:
            self.ops._ipc_close_mem(p)
        for ev in self._opened_events:
            self.ops._ipc_event_destroy(ev)
        self._opened, self._opened_events = [], []

    def close_own(self) -> None:
        """Teardown step 2, after a second barrier (every peer has run close_imports, so nobody
        maps these any more): destroy this rank's exported events and free its buffers."""
        for ev in self._events:
            self.ops._ipc_event_destroy(ev)
        self._events = []
        self._bufs = []  # the last references: hipFree through the from_blob deleter

    def close(self) -> None:
        self.close_imports()
        self.close_own()


class _HostStream:
    """One worker thread executing enqueued closures in order: the CPU model of a GPU stream."""

    def __init__(self):
        self.q: "queue.Queue[Optional[Callable[[], None]]]" = queue.Queue()
        self.error: Optional[BaseException] = None
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def _run(self):
        while True:
            fn = self.q.get()
            if fn is None:
                return
            try:
                if self.error is None:
                    fn()
            except BaseException as e:  # surfaced by synchronize()
                self.error = e

    def submit(self, fn: Callable[[], None]) -> None:
        self.q.put(fn)

    def synchronize(self, timeout: float = 120.0) -> None:
        ev = threading.Event()
        self.q.put(ev.set)
        if not ev.wait(timeout):
            raise TimeoutError("amd_dft ShmTransport: stream did not drain")
        if self.error is not None:
            raise RuntimeError("amd_dft ShmTransport: stream op failed") from self.error

    def stop(self):
        self.q.put(None)
        self.t.join(timeout=10)


class _ShmEvent:
    """Inter-process event: shared int64 ``[enqueued, completed]`` record counters."""

    def __init__(self, path: str, create: bool):
        st = torch.UntypedStorage.from_file(path, shared=True, nbytes=16)
        self.c = torch.empty(0, dtype=torch.int64).set_(st, 0, (2,))
        if create:
            self.c.zero_()
        self.path = path


class ShmTransport:
    """CPU stand-in: each buffer is a ``/dev/shm`` file mapped by every rank; pushes, event
    records and event waits run asynchronously on a per-rank worker thread (a "stream"), so the
    host runs ahead of its stream exactly as it runs ahead of a GPU."""

    def __init__(self, device: torch.device = torch.device("cpu"), spin_timeout_s: float = 120.0):
        self.device = device
        self._files: List[str] = []
        self.stream = _HostStream()
        self.spin_timeout_s = spin_timeout_s

    def _path(self) -> str:
        p = f"/dev/shm/amd_dft_ipc_{os.getpid()}_{uuid.uuid4().hex[:12]}"
        self._files.append(p)
        return p

    def alloc(self, nbytes: int):
        path = self._path()
        st = torch.UntypedStorage.from_file(path, shared=True, nbytes=nbytes)
        return torch.empty(0, dtype=torch.uint8).set_(st), (path, nbytes)

    def open(self, handle, local_buf, is_self: bool):
        if is_self:
            return local_buf
        path, nbytes = handle
        return torch.empty(0, dtype=torch.uint8).set_(torch.UntypedStorage.from_file(path, shared=True, nbytes=nbytes))

    def new_event(self):
        path = self._path()
        return _ShmEvent(path, create=True), path

    def open_event(self, handle, local_ev, is_self: bool):
        return local_ev if is_self else _ShmEvent(handle, create=False)

    def push(self, src: torch.Tensor, dsts, offset: int) -> None:
        b = src.contiguous().view(torch.uint8).reshape(-1).clone()  # snapshot at enqueue time

        def run():
            for d in dsts:
                d[offset:offset + b.numel()].copy_(b)

        self.stream.submit(run)

    def record(self, ev: _ShmEvent) -> None:
        ev.c[0] += 1
        target = int(ev.c[0])

        def run():
            ev.c[1] = target

        self.stream.submit(run)

    def wait(self, ev: _ShmEvent) -> None:
        target = int(ev.c[0])  # the peer's latest record enqueued so far (after the handshake)
        deadline_s = self.spin_timeout_s

        def run():
            t0 = time.monotonic()
            while int(ev.c[1]) < target:
                if time.monotonic() - t0 > deadline_s:
                    raise TimeoutError(f"amd_dft ShmTransport: event wait {int(ev.c[1])} < {target}")
                time.sleep(0.0005)

        self.stream.submit(run)

    def write_value(self, flags, idx: int, value: int) -> None:
        f = flags.view(torch.int32)

        def run():
            f[idx] = value

        self.stream.submit(run)

    def wait_value(self, flags, idx: int, value: int) -> None:
        f = flags.view(torch.int32)
        deadline_s = self.spin_timeout_s

        def run():
            t0 = time.monotonic()
            while int(f[idx]) < value:
                if time.monotonic() - t0 > deadline_s:
                    raise TimeoutError(f"amd_dft ShmTransport: flag wait {int(f[idx])} < {value}")
                time.sleep(0.0005)

        self.stream.submit(run)

    def enqueue(self, fn: Callable[[], None]) -> None:
        self.stream.submit(fn)

    def synchronize(self) -> None:
        self.stream.synchronize()

    def close_imports(self) -> None:
        self.stream.synchronize()
        self.stream.stop()

    def close_own(self) -> None:
        for f in self._files:
            try:
                os.unlink(f)
            except OSError:
                pass
        self._files = []

    def close(self) -> None:
        self.close_imports()
        self.close_own()


class IpcAllGather:
    """All-gather of a fixed-shape shard along dim 0 by direct pushes (see module docstring).

    ``gather(local, i)`` returns slot ``i``'s ``[world * shard_shape[0], ...]`` tensor, complete
    in stream order.  Collective: every rank constructs it with the same arguments.
    ``release=False`` drops steps 1-3 of the protocol (tests only: shows the write-after-read race).
    """

    def __init__(self, shard_shape: Sequence[int], dtype: torch.dtype, device: torch.device, *, nbuf: int = 2,
                 transport=None, group=None, release: bool = True, protocol: str = "events"):
        if protocol not in ("flags", "events"):
            raise ValueError(f"protocol must be 'flags' or 'events', not {protocol!r}")
        self.protocol = protocol
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.shard_shape = list(shard_shape)
        self.dtype = dtype
        self.nbuf = nbuf
        self.device = device
        self.release = release
        self.transport = transport or (HipIpcTransport(device) if device.type == "cuda" else ShmTransport())
        # host-side handshake group: Gloo never waits for the GPU
        self.host_group = group if group is not None else (
            dist.new_group(backend="gloo") if dist.get_backend() != "gloo" else dist.group.WORLD)
        elem = torch.empty(0, dtype=dtype).element_size()
        self.shard_bytes = int(torch.Size(self.shard_shape).numel()) * elem
        full_shape = [self.world * self.shard_shape[0]] + self.shard_shape[1:]
        self.full: List[torch.Tensor] = []
        self.peers: List[List[object]] = []
        self.events: List[object] = []      # done[i]: this rank's pushes into slot i are enqueued before it
        self.peer_events: List[List[object]] = []
        self.rel: List[object] = []         # rel[i]: this rank no longer reads its slot i
        self.peer_rel: List[List[object]] = []
        for _ in range(nbuf):
            buf, handle = self.transport.alloc(self.world * self.shard_bytes)
            ev, ev_handle = self.transport.new_event()
            rel, rel_handle = self.transport.new_event()
            handles: List[Optional[object]] = [None] * self.world
            dist.all_gather_object(handles, (handle, ev_handle, rel_handle), group=self.host_group)
            self.full.append(buf.view(dtype).view(full_shape))
            self.peers.append([self.transport.open(h[0], buf, p == self.rank) for p, h in enumerate(handles)])
            self.events.append(ev)
            self.peer_events.append([self.transport.open_event(h[1], ev, p == self.rank) for p, h in enumerate(handles)])
            self.rel.append(rel)
            self.peer_rel.append([self.transport.open_event(h[2], rel, p == self.rank) for p, h in enumerate(handles)])
        # flag words [nbuf][REL, DONE][writer rank] (int32, zeroed), written by the peers
        self.uses = [0] * nbuf
        self.flags = None
        self.peer_flags: List[object] = []
        if protocol == "flags":
            fbuf, fh = self.transport.alloc(nbuf * 2 * self.world * 4)
            fbuf.zero_()
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            fhandles: List[Optional[object]] = [None] * self.world
            dist.all_gather_object(fhandles, fh, group=self.host_group)
            self.peer_flags = [self.transport.open(h, fbuf, p == self.rank) for p, h in enumerate(fhandles)]
            self.flags = self.peer_flags[self.rank]
        dist.barrier(group=self.host_group)
        self._closed = False

    def _fi(self, slot: int, kind: int, writer: int) -> int:
        return (slot * 2 + kind) * self.world + writer

    def gather(self, local: torch.Tensor, i: int) -> torch.Tensor:
        if list(local.shape) != self.shard_shape or local.dtype != self.dtype:
            raise ValueError(f"shard {list(local.shape)} {local.dtype} != {self.shard_shape} {self.dtype}")
        i %= self.nbuf
        t = self.transport
        if self.protocol == "flags":
            self.uses[i] += 1
            n = self.uses[i]
            peers = [p for p in range(self.world) if p != self.rank]
            if self.release:
                for p in peers:
                    t.write_value(self.peer_flags[p], self._fi(i, 0, self.rank), n)
                for p in peers:
                    t.wait_value(self.flags, self._fi(i, 0, p), n)
            t.push(local, self.peers[i], self.rank * self.shard_bytes)
            for p in peers:
                t.write_value(self.peer_flags[p], self._fi(i, 1, self.rank), n)
            for p in peers:
                t.wait_value(self.flags, self._fi(i, 1, p), n)
            return self.full[i]
        if self.release:
            t.record(self.rel[i])
            dist.barrier(group=self.host_group)
            for p in range(self.world):
                if p != self.rank:
                    t.wait(self.peer_rel[i][p])
        t.push(local, self.peers[i], self.rank * self.shard_bytes)
        t.record(self.events[i])
        dist.barrier(group=self.host_group)
        for p in range(self.world):
            if p != self.rank:
                t.wait(self.peer_events[i][p])
        return self.full[i]

    def enqueue(self, fn: Callable[[], None]) -> None:
        """Run ``fn`` in this rank's stream order (CPU transport: on its worker; GPU: now)."""
        self.transport.enqueue(fn)

    def synchronize(self) -> None:
        self.transport.synchronize()

    def close(self) -> None:
        """Collective, two phases: drain this rank's stream and barrier (no push into or read of
        any buffer is in flight anywhere); every rank unmaps its peers' buffers and releases the
        peer events it opened; barrier again (nobody maps anything exported any more); only then
        does each rank destroy its own events and free its own buffers."""
        if self._closed:
            return
        self.transport.synchronize()
        dist.barrier(group=self.host_group)
        self.transport.close_imports()
        self.peers, self.peer_events, self.peer_rel, self.peer_flags, self.flags = [], [], [], [], None
        dist.barrier(group=self.host_group)
        self.full, self.events, self.rel = [], [], []
        self.transport.close_own()
        self._closed = True
