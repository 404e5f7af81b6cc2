"""Micro-batch stream parallelism inside one GPU.

FourCastNet's forward alternates MFMA-bound GEMMs (hipBLASLt, ~60 % of the time) with
memory/VALU-bound spectral kernels (FFTs, AFNO filter, LayerNorms).  Splitting the batch into
``n`` micro-batches that run the whole forward on their own HIP streams lets the hardware
dispatcher place one micro-batch's bandwidth-bound kernels on the CUs the other's GEMM is not
using (and fill each kernel's tail), instead of running every kernel alone on the chip.
Fork/join is expressed with stream waits, so the whole thing captures into one hipGraph.

Caveat: this generic wrapper lets two micro-batches' GEMMs run at the same time.  hipBLASLt's
stream-K kernels spin-wait on partial tiles of their own grid; two of them sharing the chip
can starve each other (observed: a hang at FourCastNet batch 32).  AFNONet therefore has its
own micro-batched block loop that chains the GEMMs with events (``AFNONet.micro_batches``);
use this wrapper only for modules without spinning kernels.
"""
from __future__ import annotations

from typing import List, Optional

import torch


class MicroBatchStreams(torch.nn.Module):
    def __init__(self, module: torch.nn.Module, n_streams: int = 2):
        super().__init__()
        self.module = module
        self.n = max(1, int(n_streams))
        self._streams: Optional[List[torch.cuda.Stream]] = None

    def _get_streams(self, dev: torch.device) -> List[torch.cuda.Stream]:
        if self._streams is None:
            self._streams = [torch.cuda.Stream(dev) for _ in range(self.n)]
        return self._streams

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        n = min(self.n, x.shape[0])
        if n <= 1 or x.device.type != "cuda":
            return self.module(x)
        cur = torch.cuda.current_stream(x.device)
        streams = self._get_streams(x.device)[:n]
        outs = []
        for s, xc in zip(streams, x.chunk(n)):
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                outs.append(self.module(xc))
        for s, o in zip(streams, outs):
            cur.wait_stream(s)
            o.record_stream(cur)
        return torch.cat(outs, 0)
