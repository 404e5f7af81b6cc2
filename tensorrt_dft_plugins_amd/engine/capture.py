"""hipGraph capture of an ``nn.Module`` forward with static shapes (no ONNX round trip).

Used by the benchmark and the data-parallel runner: the whole per-step forward (hundreds of
kernels: FFT passes, fused spectral kernels, GEMMs, LayerNorms) is replayed as one graph, so
launch overhead disappears (MI355X_MICROARCH.md: graph replay is one host call per step).
``n_graphs > 1`` captures several copies that write distinct output buffers but share one
memory pool, so an output can be consumed (e.g. all-gathered on another stream) while the
next step computes into the other buffer.
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
            pool = None
            for _ in range(n_graphs):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool):
                    out = self._as_list(module(*self.inputs))
                pool = g.pool()
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
