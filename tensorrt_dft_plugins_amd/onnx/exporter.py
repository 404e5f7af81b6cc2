"""PyTorch -> ONNX export with the ONNX-Runtime contrib ``Rfft`` / ``Irfft`` nodes.

Reference: the test-side autograd Functions ``OnnxRfft2`` / ``OnnxIrfft2`` whose
``symbolic`` emits ``com.microsoft::Rfft``/``Irfft`` with ``normalized_i=0, onesided_i=1,
signal_ndim_i=2`` (/root/reference/tests/test_dft.py:35-60) and the export helper
(``torch.onnx.export`` opset 15, :73-86).  Here those Functions are library API, their
``forward`` runs the MI355X kernels (``torch.ops.amd_dft``) instead of ``torch.fft``, they
cover signal_ndim 1..3, and direct calls to ``torch.ops.amd_dft.Rfft/Irfft`` export too
(custom-op symbolics).

torch 2.10's TorchScript exporter calls ``_add_onnxscript_fn``, which imports the ``onnx``
package only to splice onnx-script functions into the ModelProto; with no such functions the
pass is the identity, so :func:`export` bypasses it (the ``onnx`` package is not installed).
"""
from __future__ import annotations

import contextlib
import io
import warnings
from typing import Any, Optional, Sequence

import torch

from .._loader import load_plugins

CONTRIB_DOMAIN = "com.microsoft"
AMD_DOMAIN = "com.amd.dft"
DEFAULT_OPSET = 15


# ----------------------------------------------------------------- autograd Functions
class Rfft(torch.autograd.Function):
    """``com.microsoft::Rfft`` over the last ``signal_ndim`` dims."""

    @staticmethod
    def forward(ctx, x: torch.Tensor, signal_ndim: int = 2) -> torch.Tensor:
        load_plugins()
        return torch.ops.amd_dft.Rfft(x, 0, 1, signal_ndim)

    @staticmethod
    def symbolic(g, x, signal_ndim: int = 2):
        return g.op(f"{CONTRIB_DOMAIN}::Rfft", x, normalized_i=0, onesided_i=1, signal_ndim_i=signal_ndim)


class Irfft(torch.autograd.Function):
    """``com.microsoft::Irfft`` over the last ``signal_ndim`` dims (input has a trailing 2)."""

    @staticmethod
    def forward(ctx, x: torch.Tensor, signal_ndim: int = 2) -> torch.Tensor:
        load_plugins()
        return torch.ops.amd_dft.Irfft(x, 0, 1, signal_ndim)

    @staticmethod
    def symbolic(g, x, signal_ndim: int = 2):
        return g.op(f"{CONTRIB_DOMAIN}::Irfft", x, normalized_i=0, onesided_i=1, signal_ndim_i=signal_ndim)


class OnnxRfft2(torch.autograd.Function):
    """Drop-in for the reference test helper ``OnnxRfft2`` (signal_ndim=2)."""

    @staticmethod
    def forward(ctx, x):
        load_plugins()
        return torch.ops.amd_dft.Rfft(x, 0, 1, 2)

    @staticmethod
    def symbolic(g, x):
        return g.op(f"{CONTRIB_DOMAIN}::Rfft", x, normalized_i=0, onesided_i=1, signal_ndim_i=2)


class OnnxIrfft2(torch.autograd.Function):
    """Drop-in for the reference test helper ``OnnxIrfft2`` (signal_ndim=2)."""

    @staticmethod
    def forward(ctx, x):
        load_plugins()
        return torch.ops.amd_dft.Irfft(x, 0, 1, 2)

    @staticmethod
    def symbolic(g, x):
        return g.op(f"{CONTRIB_DOMAIN}::Irfft", x, normalized_i=0, onesided_i=1, signal_ndim_i=2)


def rfft(x: torch.Tensor, signal_ndim: int = 2) -> torch.Tensor:
    return Rfft.apply(x, signal_ndim)


def irfft(x: torch.Tensor, signal_ndim: int = 2) -> torch.Tensor:
    return Irfft.apply(x, signal_ndim)


# ----------------------------------------------------------------- custom-op symbolics
_registered: set[int] = set()


def _const_int(v) -> int:
    from torch.onnx import symbolic_helper as sh

    return int(sh._get_const(v, "i", "attr"))


def _sym_rfft(g, x, normalized, onesided, signal_ndim):
    return g.op(f"{CONTRIB_DOMAIN}::Rfft", x, normalized_i=_const_int(normalized),
                onesided_i=_const_int(onesided), signal_ndim_i=_const_int(signal_ndim))


def _sym_irfft(g, x, normalized, onesided, signal_ndim):
    return g.op(f"{CONTRIB_DOMAIN}::Irfft", x, normalized_i=_const_int(normalized),
                onesided_i=_const_int(onesided), signal_ndim_i=_const_int(signal_ndim))


_EXTRA_SYMBOLICS: dict[str, Any] = {}


def register_symbolic(qualname: str, fn) -> None:
    """Register an ONNX symbolic for another ``torch.ops.amd_dft`` operator (spectral ops)."""
    _EXTRA_SYMBOLICS[qualname] = fn


def register_symbolics(opset_version: int = DEFAULT_OPSET) -> None:
    load_plugins()
    if opset_version in _registered:
        return
    torch.onnx.register_custom_op_symbolic("amd_dft::Rfft", _sym_rfft, opset_version)
    torch.onnx.register_custom_op_symbolic("amd_dft::Irfft", _sym_irfft, opset_version)
    for name, fn in _EXTRA_SYMBOLICS.items():
        torch.onnx.register_custom_op_symbolic(name, fn, opset_version)
    _registered.add(opset_version)


@contextlib.contextmanager
def _no_onnxscript_pass():
    from torch.onnx._internal.torchscript_exporter import onnx_proto_utils as opu

    orig = opu._add_onnxscript_fn
    opu._add_onnxscript_fn = lambda model_bytes, custom_opsets: model_bytes
    try:
        yield
    finally:
        opu._add_onnxscript_fn = orig


def export(model: torch.nn.Module, args: Any, f: Optional[str | io.BytesIO] = None, *,
           opset_version: int = DEFAULT_OPSET, input_names: Optional[Sequence[str]] = None,
           output_names: Optional[Sequence[str]] = None, dynamic_axes=None, verbose: bool = False,
           do_constant_folding: bool = True) -> bytes:
    """Export ``model`` to ONNX bytes (contrib Rfft/Irfft nodes for the DFT ops).

    Equivalent of the reference's ``export_to_onnx`` (tests/test_dft.py:73-86): TorchScript
    exporter, ``OperatorExportTypes.ONNX``, opset 15 by default.  Returns the ModelProto bytes
    and also writes them to ``f`` when given.
    """
    register_symbolics(opset_version)
    if not isinstance(args, tuple):
        args = (args,)
    buf = io.BytesIO()
    with _no_onnxscript_pass(), warnings.catch_warnings():
        warnings.simplefilter("ignore")
        torch.onnx.export(
            model, args, buf, dynamo=False, operator_export_type=torch.onnx.OperatorExportTypes.ONNX,
            opset_version=opset_version, verbose=verbose, input_names=input_names, output_names=output_names,
            dynamic_axes=dynamic_axes, do_constant_folding=do_constant_folding,
            custom_opsets={CONTRIB_DOMAIN: 1, AMD_DOMAIN: 1},
        )
    data = buf.getvalue()
    if isinstance(f, str):
        with open(f, "wb") as fh:
            fh.write(data)
    elif f is not None:
        f.write(data)
    return data
