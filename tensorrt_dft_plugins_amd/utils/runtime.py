"""Runtime helpers shared by the benchmarks, the engine and the tests.

* ``finite_checks(True)`` / ``MI_DFT_CHECK_FINITE=1``: every native op validates that its
  output is finite (SURVEY §2.9 item 11 -- the reference's enqueue always returns 0,
  /root/reference/src/dft_plugins/dft_plugins.cpp:198).  The variable sets the initial state;
  ``finite_checks`` switches the loaded library at any time (and exports the variable for
  child processes).
* ``strict_mode(True)`` / ``MI_DFT_STRICT=1``: a device op that would leave its hand kernel raises.
* ``time_fn``: device time of a callable, eager or captured into one hipGraph.
* ``env_report``: the versions / devices a benchmark line should be read against.
"""
from __future__ import annotations

import os
import platform
from typing import Callable, Dict

import torch


def finite_checks(enable: bool = True) -> bool:
    """Turn the native ops' output NaN/Inf check on or off; returns the previous setting."""
    from .._loader import load_plugins

    load_plugins()
    prev = bool(torch.ops.amd_dft.set_finite_check(bool(enable)))
    os.environ["MI_DFT_CHECK_FINITE"] = "1" if enable else "0"
    return prev


def strict_mode(enable: bool = True) -> bool:
    """Make ATen / vendor fallbacks of the device ops raise (True) or warn + count (False);
    returns the previous setting."""
    from .._loader import load_plugins

    load_plugins()
    prev = bool(torch.ops.amd_dft.set_strict(bool(enable)))
    os.environ["MI_DFT_STRICT"] = "1" if enable else "0"
    return prev


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
