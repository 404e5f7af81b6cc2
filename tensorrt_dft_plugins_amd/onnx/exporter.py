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
def _contrib_node(g, kind: str, x, signal_ndim: int):
    """The contrib node, with its output type stamped (static shape inference of §2.9 items 4-5),
    so the exporter does not warn that ``com.microsoft::Rfft`` has no shape inference."""
    out = g.op(f"{CONTRIB_DOMAIN}::{kind}", x, normalized_i=0, onesided_i=1, signal_ndim_i=signal_ndim)
    try:
        from torch.onnx import symbolic_helper as sh

        sizes = sh._get_tensor_sizes(x)
        if sizes is not None and all(d is not None for d in sizes):
            if kind == "Rfft":
                sizes = list(sizes[:-1]) + [sizes[-1] // 2 + 1, 2]
            else:
                sizes = list(sizes[:-2]) + [2 * (sizes[-2] - 1)]
            out.setType(x.type().with_sizes(sizes))
    except Exception:  # noqa: BLE001 -- best effort: the importer infers shapes anyway
        pass
    return out


class Rfft(torch.autograd.Function):
    """``com.microsoft::Rfft`` over the last ``signal_ndim`` dims."""

    @staticmethod
    def forward(ctx, x: torch.Tensor, signal_ndim: int = 2) -> torch.Tensor:
        load_plugins()
        return torch.ops.amd_dft.Rfft(x, 0, 1, signal_ndim)

    @staticmethod
    def symbolic(g, x, signal_ndim: int = 2):
        return _contrib_node(g, "Rfft", x, signal_ndim)


class Irfft(torch.autograd.Function):
    """``com.microsoft::Irfft`` over the last ``signal_ndim`` dims (input has a trailing 2)."""

    @staticmethod
    def forward(ctx, x: torch.Tensor, signal_ndim: int = 2) -> torch.Tensor:
        load_plugins()
        return torch.ops.amd_dft.Irfft(x, 0, 1, signal_ndim)

    @staticmethod
    def symbolic(g, x, signal_ndim: int = 2):
        return _contrib_node(g, "Irfft", x, signal_ndim)


class OnnxRfft2(torch.autograd.Function):
    """Drop-in for the reference test helper ``OnnxRfft2`` (signal_ndim=2)."""

    @staticmethod
    def forward(ctx, x):
        load_plugins()
        return torch.ops.amd_dft.Rfft(x, 0, 1, 2)

    @staticmethod
    def symbolic(g, x):
        return _contrib_node(g, "Rfft", x, 2)


class OnnxIrfft2(torch.autograd.Function):
    """Drop-in for the reference test helper ``OnnxIrfft2`` (signal_ndim=2)."""

    @staticmethod
    def forward(ctx, x):
        load_plugins()
        return torch.ops.amd_dft.Irfft(x, 0, 1, 2)

    @staticmethod
    def symbolic(g, x):
        return _contrib_node(g, "Irfft", x, 2)


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
    if (_const_int(normalized), _const_int(onesided)) == (0, 1):
        return _contrib_node(g, "Rfft", x, _const_int(signal_ndim))
    return g.op(f"{CONTRIB_DOMAIN}::Rfft", x, normalized_i=_const_int(normalized),
                onesided_i=_const_int(onesided), signal_ndim_i=_const_int(signal_ndim))


def _sym_irfft(g, x, normalized, onesided, signal_ndim):
    if (_const_int(normalized), _const_int(onesided)) == (0, 1):
        return _contrib_node(g, "Irfft", x, _const_int(signal_ndim))
    return g.op(f"{CONTRIB_DOMAIN}::Irfft", x, normalized_i=_const_int(normalized),
                onesided_i=_const_int(onesided), signal_ndim_i=_const_int(signal_ndim))


_EXTRA_SYMBOLICS: dict[str, Any] = {}


def register_symbolic(qualname: str, fn) -> None:
    """Register an ONNX symbolic for another ``torch.ops.amd_dft`` operator (spectral ops)."""
    _EXTRA_SYMBOLICS[qualname] = fn


_TENSOR_TYPES = ("Tensor", "Optional[Tensor]")


def amd_op_names() -> list:
    """The ``torch.ops.amd_dft`` operators that export as ``com.amd.dft`` nodes (all tensor ops
    except the contrib Rfft/Irfft, which keep the ``com.microsoft`` form)."""
    load_plugins()
    out = []
    names = sorted({n.split("::", 1)[1].split(".")[0] for n in torch._C._dispatch_get_all_op_names()
                    if n.startswith("amd_dft::")})
    for name in names:
        if name in ("Rfft", "Irfft") or name.startswith("_"):
            continue
        op = getattr(torch.ops.amd_dft, name, None)
        try:
            sc = op.default._schema
        except Exception:  # noqa: BLE001 -- not an operator overload packet
            continue
        if sc.returns and all(str(r.type) == "Tensor" for r in sc.returns) and any(
                str(a.type) in _TENSOR_TYPES for a in sc.arguments):
            out.append(name)
    return sorted(out)


def _make_amd_symbolic(opname: str):
    """Generic symbolic: tensor arguments become node inputs (absent optionals recorded in
    ``tensor_mask``), scalars/lists become attributes named after the schema arguments."""
    sc = getattr(torch.ops.amd_dft, opname).default._schema
    args = list(sc.arguments)
    nret = len(sc.returns)

    def sym(g, *vals):
        from torch.onnx import symbolic_helper as sh

        tensors, mask, attrs = [], [], {}
        for a, v in zip(args, vals):
            t = str(a.type)
            if t in _TENSOR_TYPES:
                if sh._is_none(v):
                    mask.append(0)
                else:
                    mask.append(1)
                    tensors.append(v)
            elif t == "List[int]":
                ints = [int(i) for i in sh._get_const(v, "is", a.name)]
                if ints:
                    attrs[a.name + "_i"] = ints
            elif t in ("int", "bool", "SymInt"):
                attrs[a.name + "_i"] = int(sh._get_const(v, "i", a.name))
            elif t == "float":
                attrs[a.name + "_f"] = float(sh._get_const(v, "f", a.name))
            elif t == "Optional[int]":
                attrs[a.name + "_i"] = -1 if sh._is_none(v) else int(sh._get_const(v, "i", a.name))
            else:
                raise NotImplementedError(f"amd_dft::{opname}: cannot export argument {a.name}: {t}")
        attrs["tensor_mask_i"] = mask
        outs = g.op(f"{AMD_DOMAIN}::{opname}", *tensors, outputs=nret, **attrs)
        _set_output_types(opname, args, vals, outs)
        return outs

    return sym


_SCALAR = {"Float": torch.float32, "BFloat16": torch.bfloat16, "Half": torch.float16, "Double": torch.float64,
           "Long": torch.int64, "Int": torch.int32, "Bool": torch.bool}


def _set_output_types(opname, args, vals, outs) -> None:
    """Static shape inference for com.amd.dft nodes: run the op's Meta kernel on meta tensors of
    the traced input shapes and stamp the result types on the node outputs."""
    from torch.onnx import symbolic_helper as sh

    try:
        call = []
        for a, v in zip(args, vals):
            t = str(a.type)
            if t in _TENSOR_TYPES:
                if sh._is_none(v):
                    call.append(None)
                    continue
                sizes = sh._get_tensor_sizes(v)
                st = v.type().scalarType()
                if sizes is None or any(d is None for d in sizes) or st not in _SCALAR:
                    return
                call.append(torch.empty(sizes, dtype=_SCALAR[st], device="meta"))
            elif t == "List[int]":
                call.append([int(i) for i in sh._get_const(v, "is", a.name)])
            elif t in ("int", "SymInt"):
                call.append(int(sh._get_const(v, "i", a.name)))
            elif t == "bool":
                call.append(bool(sh._get_const(v, "i", a.name)))
            elif t == "float":
                call.append(float(sh._get_const(v, "f", a.name)))
            elif t == "Optional[int]":
                call.append(None if sh._is_none(v) else int(sh._get_const(v, "i", a.name)))
        res = getattr(torch.ops.amd_dft, opname)(*call)
        res = res if isinstance(res, (tuple, list)) else (res,)
        outs_l = outs if isinstance(outs, (tuple, list)) else (outs,)
        for o, r in zip(outs_l, res):
            o.setType(o.type().with_sizes(list(r.shape)).with_dtype(r.dtype))
    except Exception:  # noqa: BLE001 -- inference is best effort; the runner infers at run time
        return


def register_symbolics(opset_version: int = DEFAULT_OPSET) -> None:
    load_plugins()
    if opset_version in _registered:
        return
    torch.onnx.register_custom_op_symbolic("amd_dft::Rfft", _sym_rfft, opset_version)
    torch.onnx.register_custom_op_symbolic("amd_dft::Irfft", _sym_irfft, opset_version)
    for name in amd_op_names():
        torch.onnx.register_custom_op_symbolic(f"amd_dft::{name}", _make_amd_symbolic(name), opset_version)
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
    # no_grad: the trace is the same graph (byte-identical export), but autograd no longer keeps every
    # intermediate for a backward pass -- a batch-32 FourCastNet trace held ~170 GB of activations
    with _no_onnxscript_pass(), warnings.catch_warnings(), torch.no_grad():
        warnings.simplefilter("ignore")
        torch.onnx.export(
            model, args, buf, dynamo=False, operator_export_type=torch.onnx.OperatorExportTypes.ONNX,
            opset_version=opset_version, verbose=verbose, input_names=input_names, output_names=output_names,
            dynamic_axes=dynamic_axes, do_constant_folding=do_constant_folding,
            # no declared custom opsets: the exporter imports exactly the domains the graph uses
            # (com.microsoft and / or com.amd.dft, version 1) -- declaring both warned about the unused one
            custom_opsets={},
        )
    data = buf.getvalue()
    if isinstance(f, str):
        with open(f, "wb") as fh:
            fh.write(data)
    elif f is not None:
        f.write(data)
    return data
