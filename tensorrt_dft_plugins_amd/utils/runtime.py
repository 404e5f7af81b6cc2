"""Runtime helpers shared by the benchmarks, the engine and the tests.

* ``finite_checks(True)`` / ``MI_DFT_CHECK_FINITE=1``: every native op validates that its
  output is finite (SURVEY §2.9 item 11 -- the reference's enqueue always returns 0,
  /root/reference/src/dft_plugins/dft_plugins.cpp:198); the C++ side reads the variable once
  at first use, so set it before the first op runs.
* ``time_fn``: device time of a callable, eager or captured into one hipGraph.
* ``env_report``: the versions / devices a benchmark line should be read against.
"""
from __future__ import annotations

import os
import platform
from typing import Callable, Dict

import torch


def finite_checks(enable: bool = True) -> None:
    os.environ["MI_DFT_CHECK_FINITE"] = "1" if enable else "0"


def check_finite(t: torch.Tensor, what: str = "tensor") -> torch.Tensor:
    if not bool(torch.isfinite(t).all()):
        raise FloatingPointError(f"{what} contains NaN/Inf")
    return t


def time_fn(fn: Callable[[], object], iters: int = 20, graph: bool = True, warmup: int = 3) -> float:
    """Microseconds per call of ``fn`` on the current device."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(warmup):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0.record()
        g.replay()
        e1.record()
    else:
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / iters


def env_report() -> Dict[str, object]:
    r: Dict[str, object] = {"python": platform.python_version(), "torch": torch.__version__,
                            "hip": getattr(torch.version, "hip", None)}
    if torch.cuda.is_available():
        p = torch.cuda.get_device_properties(0)
        r.update(device=p.name, gcn_arch=getattr(p, "gcnArchName", None), cus=p.multi_processor_count,
                 mem_gb=round(p.total_memory / 2**30, 1), n_devices=torch.cuda.device_count())
    return r
