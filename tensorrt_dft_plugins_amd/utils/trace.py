"""Observability: opt-in roctx ranges and the package logger.

The reference has no tracing (timing is left to trtexec, /root/reference/README.md:61-75) and
logs only through ``trt.Logger`` in its tests (/root/reference/tests/test_dft.py:68-70).

* ``MI_DFT_TRACE=1`` (set before the first op runs): every native op pushes a roctx range
  ``amd_dft::<op>`` (csrc/ops/trace.h) and :func:`trace_range` adds Python-level ranges
  (model blocks, engine steps).  Record with
  ``rocprofv3 --marker-trace --kernel-trace -d out -- python3 script.py``.
* ``MI_DFT_LOG=DEBUG|INFO|WARNING|...`` sets the level of the ``tensorrt_dft_plugins_amd``
  logger (default WARNING), which reports plan/engine builds, GEMM tables and fallbacks.
"""
from __future__ import annotations

import contextlib
import logging
import os
import sys

import torch

_LOGGER_NAME = "tensorrt_dft_plugins_amd"


def get_logger(name: str | None = None) -> logging.Logger:
    root = logging.getLogger(_LOGGER_NAME)
    if not getattr(root, "_mi_dft_configured", False):
        root.setLevel(os.environ.get("MI_DFT_LOG", "WARNING").upper())
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(logging.Formatter("[%(name)s %(levelname)s] %(message)s"))
        root.addHandler(h)
        root.propagate = False
        root._mi_dft_configured = True
    return root if not name else root.getChild(name)


def tracing_enabled() -> bool:
    return os.environ.get("MI_DFT_TRACE", "0") not in ("", "0")


def _roctx():
    try:
        from torch.cuda import nvtx  # backed by roctx on ROCm builds

        return nvtx
    except Exception:  # pragma: no cover - torch without the nvtx/roctx binding
        return None


@contextlib.contextmanager
def trace_range(name: str):
    """roctx range (GPU timelines) + profiler record_function (torch.profiler) when tracing."""
    if not tracing_enabled():
        yield
        return
    nv = _roctx() if torch.cuda.is_available() else None
    pushed = False
    if nv is not None:
        try:
            nv.range_push(name)
            pushed = True
        except Exception:
            pushed = False
    try:
        with torch.autograd.profiler.record_function(name):
            yield
    finally:
        if pushed:
            nv.range_pop()
