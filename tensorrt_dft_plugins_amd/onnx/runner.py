"""ONNX graph importer / executor on PyTorch-ROCm tensors.

Replaces the TensorRT ONNX parser + builder of the reference's pipeline
(/root/reference/tests/test_dft.py:89-115; trtexec in README.md:61-75).  Unknown-op lookup
mirrors TensorRT's plugin-registry fallback: ``com.microsoft::Rfft/Irfft`` resolve to the
registered creators (``torch.ops.amd_dft.Rfft/Irfft``), whose attributes are validated like
the reference creator (dft_plugins.cpp:521-543, accepted by name in any order, Q10).

Shape-like int64 values (Shape/Constant/Gather/Concat chains) are evaluated on the host, so
a graph with static input shapes runs without device->host syncs and can be captured into a
hipGraph by :mod:`tensorrt_dft_plugins_amd.engine`.
"""
from __future__ import annotations

import math
import weakref
from typing import Callable, Dict, List, Optional, Sequence

import torch
import torch.nn.functional as Fn

from .._loader import load_plugins
from . import proto as P

OpFn = Callable[..., object]
_OPS: Dict[tuple, OpFn] = {}


def op(name: str, domain: str = ""):
    def deco(fn):
        _OPS[(domain, name)] = fn
        if domain == "":
            _OPS[("ai.onnx", name)] = fn
        return fn

    return deco


def supported_ops() -> List[str]:
    return sorted(f"{d}::{n}" if d else n for d, n in _OPS if d != "ai.onnx")


def _attrs(node) -> dict:
    out = {}
    for a in node.attribute:
        t = a.type
        if t == P.ATTR_FLOAT:
            out[a.name] = a.f
        elif t == P.ATTR_INT:
            out[a.name] = a.i
        elif t == P.ATTR_STRING:
            out[a.name] = a.s.decode()
        elif t == P.ATTR_TENSOR:
            out[a.name] = P.tensor_to_torch(a.t)
        elif t == P.ATTR_FLOATS:
            out[a.name] = list(a.floats)
        elif t == P.ATTR_INTS:
            out[a.name] = list(a.ints)
        elif t == P.ATTR_STRINGS:
            out[a.name] = [s.decode() for s in a.strings]
        else:
            raise NotImplementedError(f"attribute type {t} ({a.name})")
    return out


def _is_host(x) -> bool:
    return isinstance(x, torch.Tensor) and x.device.type == "cpu"


def _ints(x) -> List[int]:
    if isinstance(x, torch.Tensor):
        if x.device.type != "cpu":
            raise RuntimeError("shape-like input lives on the device; the graph is not statically shaped")
        return [int(v) for v in x.reshape(-1).tolist()]
    return [int(v) for v in x]


_DEV_CONSTS: Dict[tuple, torch.Tensor] = {}   # small host values, by value (bounded by the graphs' constants)
_DEV_LARGE: Dict[tuple, tuple] = {}            # large host tensors, by object identity, dropped with them


def _to_dev(t: torch.Tensor, device: torch.device) -> torch.Tensor:
    """Host value -> device.  0-dim host tensors stay on the host (PyTorch treats them as
    scalars, no copy); host tensors are memoised so the copy happens during warm-up and never
    inside hipGraph capture: small ones by value; a large one (e.g. folded ScatterND indices,
    held in its graph's constants) by identity, and its device copy is released when the host
    tensor is -- i.e. with the graph that owns it (a process-global memo of large
    constants grew without bound over repeated engine builds)."""
    if t.dim() == 0 or t.device == torch.device(device):
        return t
    if t.numel() <= 4096:
        key = (str(device), t.dtype, tuple(t.shape), tuple(t.reshape(-1).tolist()))
        v = _DEV_CONSTS.get(key)
        if v is None:
            v = _DEV_CONSTS[key] = t.to(device)
        return v
    key = (str(device), id(t), t._version)
    hit = _DEV_LARGE.get(key)
    if hit is not None and hit[0]() is t:
        return hit[1]
    d = t.to(device)
    _DEV_LARGE[key] = (weakref.ref(t), d)
    weakref.finalize(t, _DEV_LARGE.pop, key, None)
    return d


def _align(a, b):
    """Put host scalars/tensors next to device tensors for arithmetic."""
    if isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor) and a.device != b.device:
        if _is_host(a):
            a = _to_dev(a, b.device)
        else:
            b = _to_dev(b, a.device)
    return a, b


def _binary(f):
    def run(attrs, a, b):
        a, b = _align(a, b)
        return f(a, b)

    return run


# ----------------------------------------------------------------- elementwise / math
for _n, _f in {"Add": torch.add, "Sub": torch.sub, "Mul": torch.mul, "Pow": torch.pow,
               "Equal": torch.eq, "Greater": torch.gt, "Less": torch.lt, "GreaterOrEqual": torch.ge,
               "LessOrEqual": torch.le, "And": torch.logical_and, "Or": torch.logical_or,
               "Max": torch.maximum, "Min": torch.minimum}.items():
    _OPS[("", _n)] = _OPS[("ai.onnx", _n)] = _binary(_f)


@op("Div")
def _div(attrs, a, b):
    a, b = _align(a, b)
    if not a.is_floating_point() and not b.is_floating_point():
        return torch.div(a, b, rounding_mode="trunc")
    return a / b


for _n, _f in {"Sqrt": torch.sqrt, "Exp": torch.exp, "Log": torch.log, "Neg": torch.neg, "Abs": torch.abs,
               "Relu": torch.relu, "Sigmoid": torch.sigmoid, "Tanh": torch.tanh, "Erf": torch.erf,
               "Sign": torch.sign, "Not": torch.logical_not, "Reciprocal": torch.reciprocal,
               "Floor": torch.floor, "Ceil": torch.ceil, "Sin": torch.sin, "Cos": torch.cos,
               "Softplus": Fn.softplus, "Identity": lambda x: x}.items():
    _OPS[("", _n)] = _OPS[("ai.onnx", _n)] = (lambda f: (lambda attrs, x: f(x)))(_f)


@op("Dropout")
def _dropout(attrs, x, *rest):
    return x


@op("Gelu")
def _gelu(attrs, x):
    return Fn.gelu(x, approximate=attrs.get("approximate", "none"))


@op("LeakyRelu")
def _leaky(attrs, x):
    return Fn.leaky_relu(x, attrs.get("alpha", 0.01))


@op("Clip")
def _clip(attrs, x, lo=None, hi=None):
    lo = attrs.get("min") if lo is None else lo
    hi = attrs.get("max") if hi is None else hi
    lo = lo.item() if isinstance(lo, torch.Tensor) else lo
    hi = hi.item() if isinstance(hi, torch.Tensor) else hi
    return torch.clamp(x, lo, hi)


@op("Where")
def _where(attrs, c, a, b):
    dev = next((t.device for t in (c, a, b) if isinstance(t, torch.Tensor) and not _is_host(t)), None)
    if dev is not None:
        # 0-dim host values stay scalars (no host->device copy, which a hipGraph capture forbids)
        c, a, b = (t.item() if isinstance(t, torch.Tensor) and _is_host(t) and t.dim() == 0 and t is not c
                   else _to_dev(t, dev) if isinstance(t, torch.Tensor) and _is_host(t) else t for t in (c, a, b))
    return torch.where(c, a, b)


@op("Cast")
def _cast(attrs, x):
    return x.to(P.onnx_dtype_to_torch(attrs["to"]))


@op("Softmax")
def _softmax(attrs, x):
    return torch.softmax(x, attrs.get("axis", -1))


# ----------------------------------------------------------------- linear algebra / nn
@op("MatMul")
def _matmul(attrs, a, b):
    return torch.matmul(a, b)


@op("Gemm")
def _gemm(attrs, a, b, c=None):
    if attrs.get("transA", 0):
        a = a.t()
    if attrs.get("transB", 0):
        b = b.t()
    y = attrs.get("alpha", 1.0) * (a @ b)
    if c is not None:
        y = y + attrs.get("beta", 1.0) * c
    return y


@op("Einsum")
def _einsum(attrs, *xs):
    return torch.einsum(attrs["equation"], *xs)


@op("Conv")
def _conv(attrs, x, w, b=None):
    nd = w.dim() - 2
    pads = attrs.get("pads", [0] * (2 * nd))
    if attrs.get("auto_pad", "NOTSET") not in ("NOTSET", "VALID"):
        raise NotImplementedError("Conv auto_pad SAME_*")
    if any(pads[i] != pads[i + nd] for i in range(nd)):
        x = Fn.pad(x, [p for i in reversed(range(nd)) for p in (pads[i], pads[i + nd])])
        pad = 0
    else:
        pad = pads[:nd]
    f = {1: Fn.conv1d, 2: Fn.conv2d, 3: Fn.conv3d}[nd]
    return f(x, w, b, stride=attrs.get("strides", 1), padding=pad, dilation=attrs.get("dilations", 1),
             groups=attrs.get("group", 1))


@op("BatchNormalization")
def _bn(attrs, x, scale, bias, mean, var):
    return Fn.batch_norm(x, mean, var, scale, bias, False, 0.0, attrs.get("epsilon", 1e-5))


@op("LayerNormalization")
def _ln(attrs, x, scale, bias=None):
    axis = attrs.get("axis", -1) % x.dim()
    return Fn.layer_norm(x, x.shape[axis:], scale, bias, attrs.get("epsilon", 1e-5))


@op("GlobalAveragePool")
def _gap(attrs, x):
    return x.mean(dim=tuple(range(2, x.dim())), keepdim=True)


# ----------------------------------------------------------------- reductions
def _reduce(fn):
    def run(attrs, x, axes=None):
        axes = attrs.get("axes") if axes is None else _ints(axes)
        keep = bool(attrs.get("keepdims", 1))
        if axes is None or len(axes) == 0:
            if attrs.get("noop_with_empty_axes", 0):
                return x
            axes = list(range(x.dim()))
        return fn(x, dim=tuple(axes), keepdim=keep)

    return run


_OPS[("", "ReduceMean")] = _OPS[("ai.onnx", "ReduceMean")] = _reduce(torch.mean)
_OPS[("", "ReduceSum")] = _OPS[("ai.onnx", "ReduceSum")] = _reduce(torch.sum)
_OPS[("", "ReduceMax")] = _OPS[("ai.onnx", "ReduceMax")] = _reduce(lambda x, dim, keepdim: torch.amax(x, dim, keepdim))
_OPS[("", "ReduceMin")] = _OPS[("ai.onnx", "ReduceMin")] = _reduce(lambda x, dim, keepdim: torch.amin(x, dim, keepdim))


# ----------------------------------------------------------------- shape ops (host-evaluable)
@op("Shape")
def _shape(attrs, x):
    s = list(x.shape)
    start, end = attrs.get("start", 0), attrs.get("end", len(s))
    return torch.tensor(s[start:end], dtype=torch.int64)


@op("Size")
def _size(attrs, x):
    return torch.tensor(x.numel(), dtype=torch.int64)


@op("Constant")
def _constant(attrs):
    if "value" in attrs:
        return attrs["value"]
    for k in ("value_float", "value_int"):
        if k in attrs:
            return torch.tensor(attrs[k])
    for k in ("value_floats", "value_ints"):
        if k in attrs:
            return torch.tensor(attrs[k])
    raise NotImplementedError("Constant without value")


@op("ConstantOfShape")
def _cos(attrs, shape):
    v = attrs.get("value", torch.zeros(1, dtype=torch.float32))
    return torch.full(_ints(shape), v.reshape(-1)[0].item(), dtype=v.dtype)


@op("Reshape")
def _reshape(attrs, x, shape):
    s = _ints(shape)
    if not attrs.get("allowzero", 0):
        s = [x.shape[i] if v == 0 else v for i, v in enumerate(s)]
    return x.reshape(s)


@op("Flatten")
def _flatten(attrs, x):
    a = attrs.get("axis", 1) % max(x.dim(), 1)
    return x.reshape(int(math.prod(x.shape[:a])), -1)


@op("Transpose")
def _transpose(attrs, x):
    perm = attrs.get("perm", list(reversed(range(x.dim()))))
    return x.permute(perm)


@op("Squeeze")
def _squeeze(attrs, x, axes=None):
    axes = attrs.get("axes") if axes is None else _ints(axes)
    if axes is None:
        return x.squeeze()
    for a in sorted([a % x.dim() for a in axes], reverse=True):
        x = x.squeeze(a)
    return x


@op("Unsqueeze")
def _unsqueeze(attrs, x, axes=None):
    axes = attrs.get("axes") if axes is None else _ints(axes)
    nd = x.dim() + len(axes)
    for a in sorted(a % nd for a in axes):
        x = x.unsqueeze(a)
    return x


@op("Concat")
def _concat(attrs, *xs):
    xs = [x for x in xs if not (isinstance(x, torch.Tensor) and x.numel() == 0 and x.dim() == 1)] or list(xs)
    dev = next((x.device for x in xs if not _is_host(x)), None)
    if dev is not None:
        xs = [_to_dev(x, dev) if _is_host(x) else x for x in xs]
    return torch.cat(xs, attrs.get("axis", 0))


@op("Split")
def _split(attrs, x, split=None):
    axis = attrs.get("axis", 0)
    split = attrs.get("split") if split is None else _ints(split)
    if split is None:
        n = attrs.get("num_outputs")
        return list(torch.chunk(x, n, axis))
    return list(torch.split(x, split, axis))


@op("Slice")
def _slice(attrs, x, starts=None, ends=None, axes=None, steps=None):
    starts = attrs.get("starts") if starts is None else _ints(starts)
    ends = attrs.get("ends") if ends is None else _ints(ends)
    axes = attrs.get("axes", list(range(len(starts)))) if axes is None else _ints(axes)
    steps = [1] * len(starts) if steps is None else _ints(steps)
    idx = [slice(None)] * x.dim()
    rev = []
    for s, e, a, st in zip(starts, ends, axes, steps):
        n = x.shape[a]
        if st < 0:
            # ONNX: negative start / end get n added, then start is clamped to [0, n-1] and end to
            # [-1, n-1], walking down (end -1 after the addition = past index 0; e.g. torch's F.pad
            # export reverses its pads list with a very negative end this way)
            s = max(0, min(n - 1, s + n if s < 0 else s))
            e = max(-1, min(n - 1, e + n if e < 0 else e))
            rev.append((a % x.dim(), list(range(s, e, st))))
            continue
        s = max(0, min(n, s + n if s < 0 else s))
        e = max(0, min(n, e + n if e < 0 else e))
        idx[a % x.dim()] = slice(s, e, st)
    x = x[tuple(idx)]
    for a, ix in rev:
        x = torch.index_select(x, a, torch.tensor(ix, dtype=torch.long, device=x.device))
    return x


@op("Gather")
def _gather(attrs, x, idx):
    axis = attrs.get("axis", 0) % x.dim()
    ishape = list(idx.shape)  # a 0-d index drops the axis (kept even when moved to the device as [1])
    if _is_host(idx) and not _is_host(x):
        idx = _to_dev(idx if idx.dim() else idx.reshape(1), x.device)  # memoised: no copy under capture
    if _is_host(x) and not _is_host(idx):
        x = _to_dev(x, idx.device)
    n = x.shape[axis]
    idx = torch.where(idx < 0, idx + n, idx)
    out = torch.index_select(x, axis, idx.reshape(-1))
    return out.reshape(list(x.shape[:axis]) + ishape + list(x.shape[axis + 1:]))


@op("ScatterND")
def _scatter_nd(attrs, x, idx, upd):
    """ONNX ScatterND (torch exports in-place slice assignment, e.g. the classic FNO's
    ``out_ft[:, :, :m1, :m2] = ...``, this way)."""
    if _is_host(idx) and not _is_host(x):
        idx = _to_dev(idx, x.device)
    if _is_host(upd) and not _is_host(x):
        upd = _to_dev(upd, x.device)
    k = idx.shape[-1]
    key = tuple(idx[..., i].long() for i in range(k))
    red = attrs.get("reduction", "none")
    out = x.clone()
    if red == "none":
        out[key] = upd.to(out.dtype)
    elif red == "add":
        out.index_put_(key, upd.to(out.dtype), accumulate=True)
    elif red == "mul":
        out[key] = out[key] * upd.to(out.dtype)
    else:
        raise NotImplementedError(f"ScatterND reduction {red}")
    return out


@op("Expand")
def _expand(attrs, x, shape):
    s = _ints(shape)
    nd = max(len(s), x.dim())
    s = [1] * (nd - len(s)) + s
    xs = [1] * (nd - x.dim()) + list(x.shape)
    return x.reshape(xs).expand([max(a, b) if b != 1 or a != 1 else 1 for a, b in zip(s, xs)])


@op("Tile")
def _tile(attrs, x, reps):
    return x.repeat(_ints(reps))


@op("Range")
def _range(attrs, start, limit, delta):
    return torch.arange(start.item(), limit.item(), delta.item(), dtype=start.dtype)


@op("Pad")
def _pad(attrs, x, pads=None, value=None, axes=None):
    pads = attrs.get("pads") if pads is None else _ints(pads)
    nd = x.dim()
    tp = []
    for i in reversed(range(nd)):
        tp += [pads[i], pads[i + nd]]
    v = 0.0 if value is None else (value.item() if isinstance(value, torch.Tensor) else value)
    return Fn.pad(x, tp, mode=attrs.get("mode", "constant"), value=v)


# ----------------------------------------------------------------- DFT ops
@op("Rfft", "com.microsoft")
def _contrib_rfft(attrs, x):
    load_plugins()
    return torch.ops.amd_dft.Rfft(x, attrs.get("normalized", 0), attrs.get("onesided", 1), attrs.get("signal_ndim", 1))


@op("Irfft", "com.microsoft")
def _contrib_irfft(attrs, x):
    load_plugins()
    return torch.ops.amd_dft.Irfft(x, attrs.get("normalized", 0), attrs.get("onesided", 1), attrs.get("signal_ndim", 1))


@op("DFT")
def _onnx_dft(attrs, x, dft_length=None, axis_in=None):
    """Standard ONNX DFT (opset 17/20): real or complex ([..., 2]) input, one axis."""
    load_plugins()
    axis = int(axis_in.item()) if axis_in is not None else attrs.get("axis", -2 if x.shape[-1] in (1, 2) else 1)
    inverse = bool(attrs.get("inverse", 0))
    onesided = bool(attrs.get("onesided", 0))
    nd = x.dim() - 1
    axis = axis % (nd + 1)
    if axis == nd:
        raise ValueError("DFT axis cannot be the trailing re/im dim")
    n = int(dft_length.item()) if dft_length is not None else x.shape[axis]
    if x.shape[-1] == 1:
        xr = x[..., 0]
        if n != xr.shape[axis]:
            xr = _resize_axis(xr, axis, n)
        if onesided and not inverse:
            return torch.ops.amd_dft.r2c(xr.contiguous(), [axis], 1.0, [], torch.float32)
        xc = torch.stack([xr.float(), torch.zeros_like(xr, dtype=torch.float32)], -1)
    else:
        xc = x if n == x.shape[axis] else _resize_axis(x, axis, n)
    y = torch.ops.amd_dft.c2c(xc.float().contiguous(), [axis], inverse, 1.0 / n if inverse else 1.0, torch.float32)
    if onesided:
        y = y.narrow(axis, 0, n // 2 + 1)
    return y


def _resize_axis(x, axis, n):
    cur = x.shape[axis]
    if n <= cur:
        return x.narrow(axis, 0, n)
    s = list(x.shape)
    s[axis] = n - cur
    return torch.cat([x, x.new_zeros(s)], axis)


def register_op(name: str, domain: str, fn: OpFn) -> None:
    """Register an implementation for a custom node (``fn(attrs, *inputs)``)."""
    _OPS[(domain, name)] = fn


# ----------------------------------------------------------------- com.amd.dft nodes
AMD_DOMAIN = "com.amd.dft"


_AMD_NODE_DENY = frozenset({"wrap_device_ptr", "wrap_host_ptr", "plan_cache_clear", "plan_cache_size", "plan_cache_pinned",
                            "fallback_counts", "fallback_reset", "fallback_note", "plugin_registry"})


def _amd_node(opname: str):
    """Executor for a ``com.amd.dft::<op>`` node written by the exporter's generic symbolic:
    rebuilds the ``torch.ops.amd_dft.<op>`` call from the schema, the node inputs and attributes."""
    from .._loader import load_plugins

    load_plugins()
    from .exporter import amd_op_names

    # Only the tensor operators the exporter can emit are executable: an ONNX file or engine
    # is untrusted input, and the library also holds runtime helpers (raw-pointer wrappers,
    # cache controls) that must never be reachable from a graph.
    if opname in _AMD_NODE_DENY or opname not in amd_op_names():
        raise NotImplementedError(f"com.amd.dft::{opname}: not an exportable tensor operator of the loaded library")
    op = getattr(torch.ops.amd_dft, opname)
    sc = op.default._schema

    def run(attrs, *inputs):
        mask = list(attrs.get("tensor_mask", []))
        it = iter(inputs)
        args, mi = [], 0
        for a in sc.arguments:
            t = str(a.type)
            if t in ("Tensor", "Optional[Tensor]"):
                present = mask[mi] if mi < len(mask) else 1
                mi += 1
                args.append(next(it) if present else None)
            elif a.name in attrs:
                v = attrs[a.name]
                if t == "bool":
                    v = bool(v)
                elif t == "Optional[int]":
                    v = None if v == -1 else int(v)
                elif t == "List[int]":
                    v = [int(i) for i in v]
                args.append(v)
            else:
                args.append(a.default_value if a.has_default_value() else ([] if t == "List[int]" else None))
        return op(*args)

    return run


# ----------------------------------------------------------------- graph
class OnnxGraph:
    """A parsed ONNX model bound to a device; ``run(*inputs)`` executes it."""

    def __init__(self, model: "P.ModelProto | bytes | str", device: Optional[torch.device] = None):
        if not isinstance(model, P.ModelProto):
            model = P.load_model(model)
        self.model = model
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        g = model.graph
        self.opsets = {o.domain: o.version for o in model.opset_import}
        self.consts: Dict[str, torch.Tensor] = {}
        for t in g.initializer:
            v = P.tensor_to_torch(t)
            self.consts[t.name] = v if (v.dtype == torch.int64 and v.numel() <= 64) else v.to(self.device)
        self.input_names = [i.name for i in g.input if i.name not in self.consts]
        self.output_names = [o.name for o in g.output]
        self.input_shapes = []
        self.input_dtypes = []
        for i in g.input:
            if i.name in self.consts:
                continue
            tt = i.type.tensor_type
            self.input_shapes.append([d.dim_value if d.HasField("dim_value") else -1 for d in tt.shape.dim])
            self.input_dtypes.append(P.onnx_dtype_to_torch(tt.elem_type) if tt.elem_type else torch.float32)
        self.nodes = []
        for n in g.node:
            key = (n.domain, n.op_type)
            if key not in _OPS and n.domain == AMD_DOMAIN:
                _OPS[key] = _amd_node(n.op_type)
            if key not in _OPS:
                raise NotImplementedError(f"ONNX op {n.domain or 'ai.onnx'}::{n.op_type} is not supported "
                                          f"(node {n.name!r}); supported: {', '.join(supported_ops())}")
            attrs = _attrs(n)
            if key == ("", "Constant") or key == ("ai.onnx", "Constant"):
                v = _constant(attrs)
                self.consts[n.output[0]] = v if (v.dtype == torch.int64 and v.numel() <= 64) or v.dim() == 0 \
                    else v.to(self.device)
                continue
            self.nodes.append((_OPS[key], attrs, list(n.input), list(n.output), n.op_type))
        self.folded = self._fold_constants()
        self._plan_frees()
        # plugin-style validation of contrib nodes at build time (creator checks)
        for _, attrs, _, _, opt in self.nodes:
            if opt in ("Rfft", "Irfft"):
                if attrs.get("normalized", 0) != 0 or attrs.get("onesided", 1) != 1 or \
                        not 1 <= attrs.get("signal_ndim", 1) <= 3:
                    raise ValueError(f"invalid {opt} attributes {attrs} (normalized=0, onesided=1, "
                                     "1<=signal_ndim<=3 required)")

    def _fold_constants(self) -> int:
        """Evaluate once, at load, every node whose inputs are all constants (initializers or
        folded outputs): e.g. the bf16x3 weight splits and LayerNorm-fold weight sums of an
        exported FourCastNet, which would otherwise re-run on every replay.  TensorRT folds the
        same way at engine build.  Constants no remaining node reads are dropped."""
        kept, folded = [], 0
        with torch.no_grad():
            for node in self.nodes:
                fn, attrs, ins, outs, _ = node
                real = [i for i in ins if i]
                if not real or not all(i in self.consts for i in real):
                    kept.append(node)
                    continue
                args = [self.consts[i] if i else None for i in ins]
                while args and args[-1] is None:
                    args.pop()
                res = fn(attrs, *args)
                res = list(res) if isinstance(res, (list, tuple)) else [res]
                for o, r in zip(outs, res):
                    self.consts[o] = r
                folded += 1
        self.nodes = kept
        used = {i for _, _, ins, _, _ in kept for i in ins if i} | set(self.output_names)
        self.consts = {k: v for k, v in self.consts.items() if k in used}
        return folded

    def _plan_frees(self) -> None:
        """Per node, the values whose last reader it is: ``run`` drops them right after the node, so
        the peak footprint is the live set rather than every intermediate of the graph (the
        unoptimised contrib FourCastNet at batch 32 holds ~1000 tensors of up to 1.6 GB)."""
        keep = set(self.output_names) | set(self.consts)
        last: Dict[str, int] = {}
        for k, (_, _, ins, outs, _) in enumerate(self.nodes):
            for i in list(ins) + list(outs):
                if i and i not in keep:
                    last[i] = k
        self._frees: List[List[str]] = [[] for _ in self.nodes]
        for name, k in last.items():
            self._frees[k].append(name)

    def run(self, *inputs: torch.Tensor) -> List[torch.Tensor]:
        if len(inputs) != len(self.input_names):
            raise ValueError(f"expected {len(self.input_names)} inputs, got {len(inputs)}")
        env: Dict[str, object] = dict(self.consts)
        for name, x in zip(self.input_names, inputs):
            env[name] = x
        for (fn, attrs, ins, outs, _), frees in zip(self.nodes, self._frees):
            args = [env[i] if i else None for i in ins]
            while args and args[-1] is None:
                args.pop()
            res = fn(attrs, *args)
            del args
            if isinstance(res, (list, tuple)):
                for o, r in zip(outs, res):
                    env[o] = r
            else:
                env[outs[0]] = res
            del res
            for name in frees:
                env.pop(name, None)
        out = []
        for o in self.output_names:
            v = env[o]
            if _is_host(v) and self.device.type != "cpu":
                v = _to_dev(v, self.device) if v.dim() else _to_dev(v.reshape(1), self.device).reshape(())
            out.append(v)
        return out

    __call__ = run
