"""hipGraph capture of an ``nn.Module`` forward with static shapes (no ONNX round trip).

Used by the benchmark and the data-parallel runner: the whole per-step forward (hundreds of
kernels: FFT passes, fused spectral kernels, GEMMs, LayerNorms) is replayed as one graph, so
launch overhead disappears (MI355X_MICROARCH.md: graph replay is one host call per step).
``n_graphs > 1`` captures several copies that write distinct output buffers, so an output can be
consumed (e.g. all-gathered on another stream) while the next step computes into the other
buffer.  Each copy has its OWN memory pool: with a shared pool, the second graph's output could be
placed in blocks the first graph uses for its intermediates (freed to the pool when its capture
ends, rewritten on every replay), so replaying graph 0 while graph 1's output is still being read
on the comm stream corrupted that output (seen as a wrong self-slot in the IPC gather test, round 5).
The price is one set of intermediates per graph -- a few GB for FourCastNet at batch 32, next to
288 GB of HBM.
"""
from __future__ import annotations

from typing import List, Sequence

import torch


class CapturedModule:
    def __init__(self, module: torch.nn.Module, example_inputs: Sequence[torch.Tensor], *, warmup: int = 2,
                 n_graphs: int = 1, use_graph: bool = True):
        self.module = module
        self.inputs: List[torch.Tensor] = [x.clone() for x in example_inputs]
        dev = self.inputs[0].device
        self.use_graph = use_graph and dev.type == "cuda"
        self.graphs: List[torch.cuda.CUDAGraph] = []
        self.outputs: List[List[torch.Tensor]] = []
        with torch.no_grad():
            if not self.use_graph:
                self.outputs = [self._as_list(module(*self.inputs)) for _ in range(n_graphs)]
                return
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                for _ in range(max(1, warmup)):
                    module(*self.inputs)
            torch.cuda.current_stream(dev).wait_stream(s)
            torch.cuda.synchronize(dev)
            for _ in range(n_graphs):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):  # private pool per graph (see the module docstring)
                    out = self._as_list(module(*self.inputs))
                self.graphs.append(g)
                self.outputs.append(out)

    @staticmethod
    def _as_list(o) -> List[torch.Tensor]:
        return list(o) if isinstance(o, (list, tuple)) else [o]

    def replay(self, i: int = 0) -> List[torch.Tensor]:
        if self.use_graph:
            self.graphs[i].replay()
        else:
            with torch.no_grad():
                outs = self._as_list(self.module(*self.inputs))
            for so, o in zip(self.outputs[i], outs):
                so.copy_(o)
        return self.outputs[i]

    def __call__(self, *inputs: torch.Tensor, i: int = 0) -> List[torch.Tensor]:
        for si, x in zip(self.inputs, inputs):
            si.copy_(x, non_blocking=True)
        return self.replay(i)
