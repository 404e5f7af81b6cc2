"""Engine-build graph optimizer: map the patterns of stock ONNX graphs onto the hand kernels.

The reference's workflow is a stock PyTorch model whose FFTs are the ONNX-contrib
``Rfft`` / ``Irfft`` functions, exported to ONNX and built into a TensorRT engine
(/root/reference/README.md:3, :57-75; /root/reference/tests/test_dft.py:35-60, :73-115).
TensorRT runs the plugins for the two DFT nodes and its own fused layers for everything else.
This module is that builder step for the MI355X engine: it rewrites the exported graph, at
``Engine.build`` time, so the recognisable spectral and MLP patterns run on this library's
kernels instead of node-by-node ATen calls:

* **AFNO filter** (FourCastNet): ``Transpose -> Rfft -> [block-diagonal complex MLP, ReLU,
  softshrink on a kept-mode window] -> Irfft -> Transpose (+ filter input) (+ residual)`` ->
  ``r2c`` along W (kept modes only) -> ``afno_spectral`` (FFT_H + MFMA block MLP + IFFT_H in one
  kernel) -> ``c2r_add`` (C2R along W with both skip additions in its store).
* **FNO spectral conv**: ``Rfft -> [any per-mode linear channel mixing on a low/high mode
  window] -> Irfft (+ Conv1x1(x)) (+ GELU)`` -> ``dftw_r2c`` (truncated DFT on MFMA) ->
  ``c2c_axis`` (pruned FFT along H) -> ``fno_mix_c2c`` (mixing inside the inverse H transform)
  -> ``fno_c2r_pw`` (inverse truncated DFT + 1x1 conv + bias + GELU).
* **LayerNorm** (the opset-15 ReduceMean/Sub/Pow/Sqrt/Div decomposition or
  ``LayerNormalization``) -> ``layer_norm`` / ``layer_norm_split`` (fp32 -> bf16x3 pair rows).
* **Linear**: ``MatMul(x, W) + b (+ erf-GELU) (+ residual)`` -> ``linear`` (bf16) or
  ``linear3`` (fp32 as bf16x3 split GEMM), with the activation, the bias and the residual in the
  GEMM epilogue and split-pair outputs between chained GEMMs.
* **Patch embedding** ``Conv(k = stride = p) -> flatten -> + pos`` -> ``patch_linear(3)``, and
  the **un-patchify head** ``MatMul -> Reshape -> Transpose -> Reshape`` -> ``linear_unpatch(3)``.
* **1x1 convolutions** (+ GELU) -> ``fno_pointwise``.

Pattern matching is structural where the structure is fixed (LayerNorm, GELU, MatMul/Add) and
*numeric* where the exporter's form is arbitrary: the spectral sub-graph between an ``Rfft`` and
its ``Irfft`` is executed on probe spectra to identify the mode window, the per-mode mixing
weights (FNO: read off by unit-vector probes of a verified-linear, mode-diagonal map) or the
roles of the AFNO MLP's weights.  Every rewrite is then **verified** before it is kept: the
matched original nodes and the replacement run on the same random inputs on the build device and
must agree to the precision of the replacing kernels; otherwise the original nodes stay.  The
report (``OptimizeReport``) lists every rewrite applied or rejected and why.
"""
from __future__ import annotations

import itertools
import math
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch

from .._loader import load_plugins
from . import proto as P
from . import runner as R
from .exporter import AMD_DOMAIN, CONTRIB_DOMAIN

# ----------------------------------------------------------------------------------------- IR


@dataclass(eq=False)
class Node:
    op: str
    domain: str
    inputs: List[str]
    outputs: List[str]
    attrs: dict
    name: str = ""

    @property
    def key(self) -> Tuple[str, str]:
        return (self.domain, self.op)

    def is_(self, op: str, domain: str = "") -> bool:
        return self.op == op and (self.domain or "") in ((domain,) if domain else ("", "ai.onnx"))


@dataclass
class OptimizeReport:
    applied: List[dict] = field(default_factory=list)
    rejected: List[dict] = field(default_factory=list)
    nodes_before: int = 0
    nodes_after: int = 0

    def as_dict(self) -> dict:
        return {"applied": self.applied, "rejected": self.rejected, "nodes_before": self.nodes_before,
                "nodes_after": self.nodes_after}

    def count(self, kind: str) -> int:
        return sum(1 for a in self.applied if a["pattern"] == kind)


def _why(e: BaseException) -> str:
    """Rejection reason: a RewriteRejected's message, else the unexpected error's type and text
    (a shape the matcher did not foresee, a missing constant, a kernel's TORCH_CHECK inside the
    verification): the rewrite is dropped and the original nodes stay, the build continues."""
    return str(e) if isinstance(e, RewriteRejected) else f"{type(e).__name__}: {e}"


class RewriteRejected(Exception):
    pass


def _is_small_int(t: torch.Tensor) -> bool:
    return t.dtype == torch.int64 and t.numel() <= 64


class IRGraph:
    """A mutable node list over an ONNX ModelProto, with constants held as CPU tensors and the
    static shape / dtype of every value (from a meta-device dry run of the executor's ops)."""

    def __init__(self, model: "P.ModelProto", input_shapes: Sequence[Sequence[int]],
                 input_dtypes: Optional[Sequence[torch.dtype]] = None):
        load_plugins()
        self.model = model
        g = model.graph
        self.consts: Dict[str, torch.Tensor] = {t.name: P.tensor_to_torch(t) for t in g.initializer}
        self.input_names = [i.name for i in g.input if i.name not in self.consts]
        self.output_names = [o.name for o in g.output]
        dts = list(input_dtypes) if input_dtypes is not None else [
            P.onnx_dtype_to_torch(i.type.tensor_type.elem_type) if i.type.tensor_type.elem_type else torch.float32
            for i in g.input if i.name not in self.consts]
        self.input_meta = {n: (list(map(int, s)), dt) for n, s, dt in zip(self.input_names, input_shapes, dts)}
        self.nodes: List[Node] = []
        for i, n in enumerate(g.node):
            attrs = R._attrs(n)
            if n.op_type == "Constant" and (n.domain or "") in ("", "ai.onnx"):
                self.consts[n.output[0]] = R._constant(attrs)
                continue
            self.nodes.append(Node(n.op_type, n.domain or "", list(n.input), list(n.output), attrs,
                                   n.name or f"n{i}"))
        self.meta: Dict[str, Tuple[List[int], torch.dtype]] = {}
        # fp32 originals of the split-pair weight constants the rewrites create (build-time only,
        # never serialised): later passes re-derive operands from them without the split's rounding
        self.orig: Dict[str, torch.Tensor] = {}
        self._uid = 0

    # ------------------------------------------------------------------ bookkeeping
    def fresh(self, stem: str) -> str:
        self._uid += 1
        return f"amdopt::{stem}_{self._uid}"

    def producers(self) -> Dict[str, Node]:
        return {o: n for n in self.nodes for o in n.outputs if o}

    def consumers(self) -> Dict[str, List[Node]]:
        out: Dict[str, List[Node]] = {}
        for n in self.nodes:
            for i in n.inputs:
                if i:
                    out.setdefault(i, []).append(n)
        return out

    def const(self, name: str) -> Optional[torch.Tensor]:
        return self.consts.get(name) if name else None

    def scalar(self, name: str) -> Optional[float]:
        c = self.const(name)
        if c is None or c.numel() != 1 or not (c.is_floating_point() or c.dtype in (torch.int64, torch.int32)):
            return None
        return float(c.reshape(-1)[0])

    def shape(self, name: str) -> Optional[List[int]]:
        m = self.meta.get(name)
        return None if m is None else m[0]

    def dtype(self, name: str) -> Optional[torch.dtype]:
        m = self.meta.get(name)
        return None if m is None else m[1]

    def add_const(self, stem: str, t: torch.Tensor) -> str:
        name = self.fresh(stem)
        self.consts[name] = t.detach().cpu().contiguous()
        self.meta[name] = (list(t.shape), t.dtype)
        return name

    # ------------------------------------------------------------------ passes
    def _fn(self, n: Node):
        if n.key not in R._OPS and n.domain == AMD_DOMAIN:
            R._OPS[n.key] = R._amd_node(n.op)
        fn = R._OPS.get(n.key) or R._OPS.get(("", n.op) if n.domain in ("", "ai.onnx") else n.key)
        if fn is None:
            raise NotImplementedError(f"{n.domain}::{n.op}")
        return fn

    def fold_constants(self) -> int:
        """Evaluate (on the CPU, once) every node whose inputs are all constants."""
        kept, folded = [], 0
        with torch.no_grad():
            for n in self.nodes:
                real = [i for i in n.inputs if i]
                if not real or not all(i in self.consts for i in real) or n.domain == CONTRIB_DOMAIN:
                    kept.append(n)
                    continue
                args = [self.consts[i] if i else None for i in n.inputs]
                while args and args[-1] is None:
                    args.pop()
                res = self._fn(n)(n.attrs, *args)
                res = list(res) if isinstance(res, (list, tuple)) else [res]
                for o, r in zip(n.outputs, res):
                    self.consts[o] = r.cpu() if isinstance(r, torch.Tensor) else torch.tensor(r)
                folded += 1
        self.nodes = kept
        return folded

    def fold_shapes(self) -> int:
        """Shape / Size of a statically shaped value -> constant (then foldable downstream)."""
        kept, n_f = [], 0
        for n in self.nodes:
            src = n.inputs[0] if n.inputs else ""
            if (n.is_("Shape") or n.is_("Size")) and src in self.meta:
                s = self.meta[src][0]
                if n.is_("Shape"):
                    a, b = n.attrs.get("start", 0), n.attrs.get("end", len(s))
                    self.consts[n.outputs[0]] = torch.tensor(s[a:b], dtype=torch.int64)
                else:
                    self.consts[n.outputs[0]] = torch.tensor(int(math.prod(s)), dtype=torch.int64)
                n_f += 1
                continue
            kept.append(n)
        self.nodes = kept
        return n_f

    def eliminate_noops(self) -> int:
        """Drop Identity nodes and Casts to the dtype the value already has (renaming consumers)."""
        outs = set(self.output_names)
        ren: Dict[str, str] = {}
        kept = []
        for n in self.nodes:
            src = ren.get(n.inputs[0], n.inputs[0]) if n.inputs else None
            noop = n.is_("Identity") or (n.is_("Cast") and self.dtype(src) is not None
                                         and P.onnx_dtype_to_torch(n.attrs["to"]) == self.dtype(src))
            if noop and n.outputs[0] not in outs:
                ren[n.outputs[0]] = src
                continue
            n.inputs = [ren.get(i, i) for i in n.inputs]
            kept.append(n)
        self.nodes = kept
        return len(ren)

    def dead_code(self) -> None:
        live = set(self.output_names)
        kept = []
        for n in reversed(self.nodes):
            if any(o in live for o in n.outputs):
                kept.append(n)
                live.update(i for i in n.inputs if i)
        self.nodes = list(reversed(kept))
        self.consts = {k: v for k, v in self.consts.items() if k in live}

    def infer_shapes(self) -> None:
        """Static shapes/dtypes of every value: run the executor's ops on meta tensors."""
        env: Dict[str, object] = {}
        for k, v in self.consts.items():
            env[k] = v if _is_small_int(v) or v.dim() == 0 else torch.empty(v.shape, dtype=v.dtype, device="meta")
            self.meta[k] = (list(v.shape), v.dtype)
        for name, (s, dt) in self.input_meta.items():
            env[name] = torch.empty(s, dtype=dt, device="meta")
            self.meta[name] = (s, dt)
        with torch.no_grad():
            for n in self.nodes:
                if not all((not i) or i in env for i in n.inputs):
                    continue
                args = [env[i] if i else None for i in n.inputs]
                while args and args[-1] is None:
                    args.pop()
                try:
                    res = self._fn(n)(n.attrs, *args)
                except Exception:  # noqa: BLE001 -- an op without a meta path: its consumers stay unknown
                    continue
                res = list(res) if isinstance(res, (list, tuple)) else [res]
                for o, r in zip(n.outputs, res):
                    if isinstance(r, torch.Tensor):
                        env[o] = r
                        self.meta[o] = (list(r.shape), r.dtype)

    # ------------------------------------------------------------------ execution (verification)
    def run_nodes(self, nodes: Iterable[Node], env: Dict[str, object], device) -> Dict[str, object]:
        env = dict(env)
        with torch.no_grad():
            for n in nodes:
                args = []
                for i in n.inputs:
                    if not i:
                        args.append(None)
                    elif i in env:
                        args.append(env[i])
                    else:
                        c = self.consts[i]
                        args.append(c if _is_small_int(c) or c.dim() == 0 else c.to(device))
                while args and args[-1] is None:
                    args.pop()
                res = self._fn(n)(n.attrs, *args)
                res = list(res) if isinstance(res, (list, tuple)) else [res]
                for o, r in zip(n.outputs, res):
                    env[o] = r
        return env

    # ------------------------------------------------------------------ output
    def to_model(self) -> "P.ModelProto":
        m = P.ModelProto()
        m.CopyFrom(self.model)
        g = m.graph
        del g.node[:]
        del g.initializer[:]
        used = {i for n in self.nodes for i in n.inputs if i} | set(self.output_names)
        keep_inputs = [vi for vi in self.model.graph.input if vi.name in self.input_meta]
        del g.input[:]
        for vi in keep_inputs:
            g.input.add().CopyFrom(vi)
        del g.value_info[:]
        for k, v in self.consts.items():
            if k in used:
                g.initializer.add().CopyFrom(P.torch_to_tensor(v, k))
        for n in self.nodes:
            pn = g.node.add()
            pn.op_type, pn.domain, pn.name = n.op, n.domain, n.name
            pn.input.extend(n.inputs)
            pn.output.extend(n.outputs)
            for k, v in n.attrs.items():
                _set_attr(pn.attribute.add(), k, v)
        if not any(o.domain == AMD_DOMAIN for o in m.opset_import):
            op = m.opset_import.add()
            op.domain, op.version = AMD_DOMAIN, 1
        return m


def _set_attr(a, name: str, v) -> None:
    a.name = name
    if isinstance(v, bool) or isinstance(v, int):
        a.type, a.i = P.ATTR_INT, int(v)
    elif isinstance(v, float):
        a.type, a.f = P.ATTR_FLOAT, v
    elif isinstance(v, str):
        a.type, a.s = P.ATTR_STRING, v.encode()
    elif isinstance(v, torch.Tensor):
        a.type = P.ATTR_TENSOR
        a.t.CopyFrom(P.torch_to_tensor(v))
    elif isinstance(v, (list, tuple)) and all(isinstance(x, (int, bool)) for x in v):
        a.type = P.ATTR_INTS
        a.ints.extend(int(x) for x in v)
    elif isinstance(v, (list, tuple)) and all(isinstance(x, (int, float)) for x in v):
        a.type = P.ATTR_FLOATS
        a.floats.extend(float(x) for x in v)
    elif isinstance(v, (list, tuple)) and all(isinstance(x, str) for x in v):
        a.type = P.ATTR_STRINGS
        a.strings.extend(x.encode() for x in v)
    else:
        raise TypeError(f"attribute {name}: cannot encode {type(v)}")


_SCALARTYPE = {torch.float32: 6, torch.bfloat16: 15, torch.float16: 5}


def amd_node(g: IRGraph, opname: str, tensors: Sequence[Optional[str]], outputs: Sequence[str], **scalars) -> Node:
    """A ``com.amd.dft::<op>`` node in the exporter's encoding (tensor inputs + ``tensor_mask``,
    scalar schema arguments as attributes), runnable by the executor and serialisable."""
    op = getattr(torch.ops.amd_dft, opname)
    sc = op.default._schema
    tensor_args = [a for a in sc.arguments if str(a.type) in ("Tensor", "Optional[Tensor]")]
    if len(tensors) > len(tensor_args):
        raise ValueError(f"{opname}: {len(tensors)} tensors for {len(tensor_args)} tensor args")
    tensors = list(tensors) + [None] * (len(tensor_args) - len(tensors))
    attrs: dict = {"tensor_mask": [0 if t is None else 1 for t in tensors]}
    names = {a.name for a in sc.arguments}
    for k, v in scalars.items():
        if k not in names:
            raise ValueError(f"{opname}: no argument {k}")
        if isinstance(v, torch.dtype):
            v = _SCALARTYPE[v]
        attrs[k] = v
    return Node(opname, AMD_DOMAIN, [t for t in tensors if t is not None], list(outputs), attrs, g.fresh(opname))


# ----------------------------------------------------------------------------------------- matching helpers


class Ctx:
    def __init__(self, g: IRGraph, device: torch.device, report: OptimizeReport, verify: bool = True, progress=None):
        self.g, self.device, self.report, self.verify = g, device, report, verify
        self.progress = progress
        self.refresh()

    def refresh(self) -> None:
        self.prod = self.g.producers()
        self.cons = self.g.consumers()

    def producer(self, v: str, op: Optional[str] = None) -> Optional[Node]:
        n = self.prod.get(v)
        if n is None or (op is not None and not n.is_(op)):
            return None
        return n

    def only_consumer(self, v: str, op: Optional[str] = None) -> Optional[Node]:
        c = self.cons.get(v, [])
        if len(c) != 1 or v in self.g.output_names:
            return None
        if op is not None and not c[0].is_(op):
            return None
        return c[0]

    def other_input(self, n: Node, v: str) -> Optional[str]:
        ins = [i for i in n.inputs if i]
        if len(ins) != 2 or v not in ins:
            return None
        return ins[1] if ins[0] == v else ins[0]

    def replace(self, old: Sequence[Node], new: Sequence[Node], outputs_map: Dict[str, str]) -> None:
        """Remove ``old``, insert ``new`` where the first removed node was, rename values."""
        ids = {id(n) for n in old}
        # a graph output keeps its name: the replacement's value is renamed to it instead
        keep = {v: k for k, v in outputs_map.items() if k in self.g.output_names}
        if keep:
            for n in new:
                n.outputs = [keep.get(o, o) for o in n.outputs]
                n.inputs = [keep.get(i, i) for i in n.inputs]
            for v, k in keep.items():
                if v in self.g.meta:
                    self.g.meta[k] = self.g.meta[v]
            outputs_map = {k: v for k, v in outputs_map.items() if k not in keep.values()}
        pos = min(i for i, n in enumerate(self.g.nodes) if id(n) in ids)
        rest = [n for n in self.g.nodes if id(n) not in ids]
        before = sum(1 for n in self.g.nodes[:pos] if id(n) not in ids)
        self.g.nodes = rest[:before] + list(new) + rest[before:]
        if outputs_map:
            for n in self.g.nodes:
                n.inputs = [outputs_map.get(i, i) for i in n.inputs]
            self.g.output_names = [outputs_map.get(o, o) for o in self.g.output_names]
        self.refresh()

    def topo_fix(self) -> None:
        """Re-sort nodes topologically (a replacement may read a value defined later)."""
        have = set(self.g.consts) | set(self.g.input_names)
        pending = list(self.g.nodes)
        out = []
        while pending:
            progress = False
            rest = []
            for n in pending:
                if all((not i) or i in have for i in n.inputs):
                    out.append(n)
                    have.update(o for o in n.outputs if o)
                    progress = True
                else:
                    rest.append(n)
            pending = rest
            if not progress:
                miss = sorted({i for n in pending for i in n.inputs if i and i not in have})[:8]
                raise RuntimeError(f"graph has a cycle after rewriting (unresolved inputs {miss})")
        self.g.nodes = out
        self.refresh()


def _rel(a: torch.Tensor, b: torch.Tensor) -> float:
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _gen(device, seed: int) -> torch.Generator:
    """A generator on the build device: full-size probes are drawn there, not on the host."""
    return torch.Generator(device=device).manual_seed(seed)


def _rand_for(g: IRGraph, name: str, device, gen: torch.Generator, scale: float = 1.0) -> torch.Tensor:
    s, dt = g.meta[name]
    return (torch.randn(s, generator=gen, dtype=torch.float32, device=device) * scale).to(dtype=dt)


def _verify(ctx: Ctx, old: Sequence[Node], new: Sequence[Node], ins: Sequence[str], outs_old: Sequence[str],
            outs_new: Sequence[str], tol: float, scales: Sequence[float] = (1.0,)) -> float:
    """Run the original nodes and the replacement on the same random boundary inputs; return the
    worst relative L2 difference (raises RewriteRejected above ``tol``)."""
    if not ctx.verify:
        return float("nan")
    g = ctx.g
    worst = 0.0
    for si, sc in enumerate(scales):
        gen = _gen(ctx.device, 1234 + si)
        env = {i: _rand_for(g, i, ctx.device, gen, sc) for i in ins}
        e1 = g.run_nodes(old, env, ctx.device)
        e2 = g.run_nodes(new, env, ctx.device)
        for a, b in zip(outs_old, outs_new):
            r = _rel(e2[b].float(), e1[a].float())
            if not math.isfinite(r) or r > tol:
                raise RewriteRejected(f"verification failed: rel-L2 {r:.3g} > {tol:g} (input scale {sc})")
            worst = max(worst, r)
    return worst


def _precision_tol(dt: torch.dtype) -> float:
    return 3e-2 if dt == torch.bfloat16 else 1e-4


# ----------------------------------------------------------------------------------------- patterns
def _gelu_after(ctx: Ctx, v: str) -> Optional[Tuple[List[Node], str]]:
    """erf-GELU of ``v`` in torch's export form: Div(v, sqrt2) | Mul(v, 1/sqrt2) -> Erf ->
    Add(., 1) -> Mul(v, .) -> Mul(., 0.5) (operand orders free).  Returns (nodes, output)."""
    cons = ctx.cons.get(v, [])
    if len(cons) != 2:
        return None
    d = next((n for n in cons if n.is_("Div") or n.is_("Mul")), None)
    if d is None or d.inputs[0] != v and d.is_("Div"):
        return None
    c = ctx.g.scalar(ctx.other_input(d, v) or "")
    if c is None or not (abs(c - math.sqrt(2)) < 1e-3 if d.is_("Div") else abs(c - 1 / math.sqrt(2)) < 1e-3):
        return None
    erf = ctx.only_consumer(d.outputs[0], "Erf")
    if erf is None:
        return None
    a1 = ctx.only_consumer(erf.outputs[0], "Add")
    if a1 is None or ctx.g.scalar(ctx.other_input(a1, erf.outputs[0]) or "") != 1.0:
        return None
    m1 = ctx.only_consumer(a1.outputs[0], "Mul")
    if m1 is None or ctx.other_input(m1, a1.outputs[0]) != v or m1 not in cons:
        return None
    m2 = ctx.only_consumer(m1.outputs[0], "Mul")
    if m2 is None or ctx.g.scalar(ctx.other_input(m2, m1.outputs[0]) or "") != 0.5:
        return None
    return [d, erf, a1, m1, m2], m2.outputs[0]


def rewrite_layernorm(ctx: Ctx) -> None:
    """ReduceMean/Sub/Pow/ReduceMean/Add(eps)/Sqrt/Div/Mul(gamma)/Add(beta) over the last axis, or
    LayerNormalization(axis=-1) -> amd_dft::layer_norm."""
    g = ctx.g
    for sq in [n for n in g.nodes if n.is_("Sqrt") or n.is_("LayerNormalization")]:
        if sq not in g.nodes:
            continue
        try:
            if sq.is_("LayerNormalization"):
                x, gamma = sq.inputs[0], sq.inputs[1]
                beta = sq.inputs[2] if len(sq.inputs) > 2 else ""
                eps = float(sq.attrs.get("epsilon", 1e-5))
                C = g.shape(x)[-1]
                if sq.attrs.get("axis", -1) not in (-1, len(g.shape(x)) - 1) or len(sq.outputs) > 1 and any(sq.outputs[1:]):
                    raise RewriteRejected("LayerNormalization over more than the last axis / with stats outputs")
                old, out = [sq], sq.outputs[0]
            else:
                ad = ctx.producer(sq.inputs[0], "Add")
                if ad is None:
                    continue
                rm2 = next((ctx.producer(i, "ReduceMean") for i in ad.inputs if ctx.producer(i, "ReduceMean")), None)
                if rm2 is None:
                    continue
                eps = g.scalar(ctx.other_input(ad, rm2.outputs[0]) or "")
                pw = ctx.producer(rm2.inputs[0], "Pow")
                if eps is None or pw is None or g.scalar(pw.inputs[1]) != 2.0:
                    continue
                sub = ctx.producer(pw.inputs[0], "Sub")
                if sub is None:
                    continue
                rm1 = ctx.producer(sub.inputs[1], "ReduceMean")
                x = sub.inputs[0]
                if rm1 is None or rm1.inputs[0] != x:
                    continue
                for rm in (rm1, rm2):
                    axes = rm.attrs.get("axes") or (g.consts[rm.inputs[1]].tolist() if len(rm.inputs) > 1 else None)
                    if axes is None or [a % len(g.shape(x)) for a in axes] != [len(g.shape(x)) - 1] or \
                            not rm.attrs.get("keepdims", 1):
                        raise RewriteRejected("LayerNorm reduction is not over the last axis")
                dv = ctx.only_consumer(sq.outputs[0], "Div")
                if dv is None or dv.inputs != [sub.outputs[0], sq.outputs[0]]:
                    continue
                if sorted(id(n) for n in ctx.cons.get(sub.outputs[0], [])) != sorted([id(pw), id(dv)]):
                    continue
                mu = ctx.only_consumer(dv.outputs[0], "Mul")
                C = g.shape(x)[-1]
                gamma = ctx.other_input(mu, dv.outputs[0]) if mu is not None else None
                if gamma is None or g.const(gamma) is None or g.const(gamma).numel() != C:
                    continue
                ab = ctx.only_consumer(mu.outputs[0], "Add")
                beta = ctx.other_input(ab, mu.outputs[0]) if ab is not None else None
                if beta is None or g.const(beta) is None or g.const(beta).numel() != C:
                    raise RewriteRejected("LayerNorm without a constant bias")
                old = [rm1, sub, pw, rm2, ad, sq, dv, mu, ab]
                out = ab.outputs[0]
            dt = g.dtype(x)
            gw = g.add_const("ln_w", g.consts[gamma].float().reshape(C))
            gb = g.add_const("ln_b", (g.consts[beta].float().reshape(C) if beta else torch.zeros(C)))
            y = g.fresh("ln_out")
            n = amd_node(g, "layer_norm", [x, gw, gb, None], [y, g.fresh("ln_sum")], eps=float(eps))
            g.meta[y] = (g.shape(out), g.dtype(out))
            err = _verify(ctx, old, [n], [x], [out], [y], _precision_tol(dt))
            ctx.replace(old, [n], {out: y})
            ctx.report.applied.append({"pattern": "layer_norm", "at": sq.name, "rel_l2": err})
        except Exception as e:  # noqa: BLE001 -- any failure keeps the original nodes
            ctx.report.rejected.append({"pattern": "layer_norm", "at": sq.name, "why": _why(e)})


def _gemm_ok(N: int, K: int, split: bool) -> bool:
    return N % 64 == 0 and N >= 64 and (K % 32 == 0 and K >= 64 if split else K % 64 == 0)


def rewrite_linear(ctx: Ctx) -> None:
    """MatMul(x, W[K, N] const) + b (or Gemm(x, W, b), torch's export of nn.Linear on 2-D input)
    (+ erf-GELU) (+ residual Add) -> linear (bf16) / split_bf16 + linear3 (fp32, bf16x3)."""
    g = ctx.g
    for mm in [n for n in g.nodes if n.is_("MatMul") or n.is_("Gemm")]:
        if mm not in g.nodes:
            continue
        try:
            x, wname = mm.inputs[:2]
            W = g.const(wname)
            if W is None or W.dim() != 2 or g.shape(x) is None:
                continue
            gemm_bias = None
            if mm.is_("Gemm"):
                if mm.attrs.get("transA", 0) or mm.attrs.get("alpha", 1.0) != 1.0 or mm.attrs.get("beta", 1.0) != 1.0 \
                        or len(g.shape(x)) != 2:
                    continue
                if mm.attrs.get("transB", 0):
                    W = W.t()
                if len(mm.inputs) > 2 and mm.inputs[2]:
                    gemm_bias = mm.inputs[2]
                    if g.const(gemm_bias) is None or g.const(gemm_bias).numel() != W.shape[1]:
                        continue
            K, N = W.shape
            dt = g.dtype(x)
            if dt not in (torch.float32, torch.bfloat16):
                continue
            split = dt == torch.float32
            if not _gemm_ok(N, K, split):
                raise RewriteRejected(f"hand GEMM tile constraints (N={N}, K={K})")
            old, out, bias, act, residual = [mm], mm.outputs[0], gemm_bias, 0, None
            ab = ctx.only_consumer(out, "Add") if gemm_bias is None else None
            if ab is not None:
                b = ctx.other_input(ab, out)
                if b is not None and g.const(b) is not None and g.const(b).numel() == N:
                    bias, out = b, ab.outputs[0]
                    old.append(ab)
            ge = _gelu_after(ctx, out)
            if ge is not None:
                old += ge[0]
                out, act = ge[1], 1
            else:
                ar = ctx.only_consumer(out, "Add")
                r = ctx.other_input(ar, out) if ar is not None else None
                if r is not None and g.shape(r) == g.shape(out) and g.dtype(r) == g.dtype(out) and \
                        g.const(r) is None:
                    residual, out = r, ar.outputs[0]
                    old.append(ar)
            wt = W.t().contiguous().float()
            bname = g.add_const("lin_b", g.consts[bias].float().reshape(N)) if bias else None
            y = g.fresh("lin_out")
            new = []
            if split:
                xs = g.fresh("lin_xs")
                new.append(amd_node(g, "split_bf16", [x], [xs], rows=True))
                g.meta[xs] = (g.shape(x)[:-1] + [2 * K], torch.bfloat16)
                from ..ops.spectral import split_bf16
                ws = g.add_const("lin_ws", split_bf16(wt))
                g.orig[ws] = wt
                new.append(amd_node(g, "linear3", [xs, ws, bname, residual], [y], act=act, split_out=False))
            else:
                wb = g.add_const("lin_w", wt.to(torch.bfloat16))
                new.append(amd_node(g, "linear", [x, wb, bname, residual], [y], act=act))
            g.meta[y] = (g.shape(out), g.dtype(out))
            ins = [x] + ([residual] if residual else [])
            err = _verify(ctx, old, new, ins, [out], [y], 1e-4 if split else 3e-2)
            ctx.replace(old, new, {out: y})
            ctx.report.applied.append({"pattern": "linear" + ("_gelu" if act else "") + ("_residual" if residual else ""),
                                       "at": mm.name, "rel_l2": err, "precision": "bf16x3" if split else "bf16"})
        except Exception as e:  # noqa: BLE001 -- any failure keeps the original nodes
            ctx.report.rejected.append({"pattern": "linear", "at": mm.name, "why": _why(e)})


def fuse_split_chains(ctx: Ctx) -> None:
    """Peepholes over the emitted nodes: a ``linear3`` whose output only feeds ``split_bf16``
    writes the split pairs itself (``split_out``); a ``layer_norm`` whose output only feeds
    ``split_bf16`` becomes ``layer_norm_split``."""
    g = ctx.g
    for sp in [n for n in g.nodes if n.domain == AMD_DOMAIN and n.op == "split_bf16"]:
        src = ctx.producer(sp.inputs[0])
        if src is None or src.domain != AMD_DOMAIN:
            continue
        users = ctx.cons.get(sp.inputs[0], [])
        if sp.inputs[0] in g.output_names or any(u.op != "split_bf16" for u in users):
            continue
        if src.op == "linear3" and not src.attrs.get("split_out") and src.attrs["tensor_mask"][3] == 0:
            src.attrs["split_out"] = True
        elif src.op == "layer_norm" and src.outputs[0] == sp.inputs[0] and src.attrs["tensor_mask"][3] == 0 and \
                not ctx.cons.get(src.outputs[1]):
            src.op = "layer_norm_split"
            src.attrs = {"tensor_mask": [1, 1, 1, 0], "eps": src.attrs["eps"]}
            src.outputs = [src.outputs[0]]
        else:
            continue
        ren = {}
        for u in users:
            ren[u.outputs[0]] = src.outputs[0]
        ctx.replace(users, [], ren)
        g.meta[src.outputs[0]] = g.meta.get(users[0].outputs[0], g.meta.get(src.outputs[0]))
        ctx.report.applied.append({"pattern": "split_fused_" + src.op, "at": src.name})


def rewrite_pointwise_conv(ctx: Ctx) -> None:
    """Conv 1x1 (+ erf-GELU) on [B, C, H, W] -> fno_pointwise."""
    g = ctx.g
    for cv in [n for n in g.nodes if n.is_("Conv")]:
        if cv not in g.nodes:
            continue
        W = g.const(cv.inputs[1])
        if W is None or W.dim() != 4 or tuple(W.shape[2:]) != (1, 1) or cv.attrs.get("group", 1) != 1:
            continue
        if any(s != 1 for s in cv.attrs.get("strides", [1, 1])) or any(p != 0 for p in cv.attrs.get("pads", [0] * 4)):
            continue
        x = cv.inputs[0]
        if g.dtype(x) not in (torch.float32, torch.bfloat16):
            continue
        try:
            old, out, gelu = [cv], cv.outputs[0], False
            ge = _gelu_after(ctx, out)
            if ge is not None:
                old += ge[0]
                out, gelu = ge[1], True
            wname = g.add_const("pw_w", W.reshape(W.shape[0], W.shape[1]).float())
            bname = g.add_const("pw_b", g.consts[cv.inputs[2]].float()) if len(cv.inputs) > 2 and cv.inputs[2] else None
            y = g.fresh("pw_out")
            n = amd_node(g, "fno_pointwise", [None, x, wname, bname], [y], gelu=gelu)
            g.meta[y] = (g.shape(out), g.dtype(out))
            err = _verify(ctx, old, [n], [x], [out], [y], _precision_tol(g.dtype(x)))
            ctx.replace(old, [n], {out: y})
            ctx.report.applied.append({"pattern": "pointwise_conv" + ("_gelu" if gelu else ""), "at": cv.name,
                                       "rel_l2": err})
        except Exception as e:  # noqa: BLE001 -- any failure keeps the original nodes
            ctx.report.rejected.append({"pattern": "pointwise_conv", "at": cv.name, "why": _why(e)})


def rewrite_patch_embed(ctx: Ctx) -> None:
    """Conv(k = stride = p, no pad) -> Reshape [B, N, hw] -> Transpose(0, 2, 1) -> Add(pos)
    (-> Reshape) -> patch_linear (bf16) / patch_linear3 (fp32 on split image planes)."""
    g = ctx.g
    for cv in [n for n in g.nodes if n.is_("Conv")]:
        if cv not in g.nodes:
            continue
        W = g.const(cv.inputs[1])
        if W is None or W.dim() != 4:
            continue
        p = W.shape[2]
        if W.shape[3] != p or p == 1 or cv.attrs.get("strides") != [p, p] or any(cv.attrs.get("pads", [0] * 4)):
            continue
        x = cv.inputs[0]
        try:
            if cv.attrs.get("group", 1) != 1 or any(d != 1 for d in cv.attrs.get("dilations", [1, 1])):
                raise RewriteRejected("patch embedding needs group == 1 and unit dilations")
            dt = g.dtype(x)
            if dt not in (torch.float32, torch.bfloat16) or p != 8:
                raise RewriteRejected("patch embedding needs p == 8 and fp32/bf16")
            if g.shape(x) is None or len(g.shape(x)) != 4:
                raise RewriteRejected("patch embedding input shape unknown / not 4-D")
            B, Cin, Hh, Ww = g.shape(x)
            if W.shape[1] != Cin:
                raise RewriteRejected("patch embedding weight does not span every input channel")
            N = W.shape[0]
            h, w = Hh // p, Ww // p
            if N % 64:
                raise RewriteRejected(f"patch embedding width {N} not a multiple of 64")
            rs = ctx.only_consumer(cv.outputs[0], "Reshape")
            if rs is None or g.shape(rs.outputs[0]) != [B, N, h * w]:
                raise RewriteRejected("conv output is not flattened to [B, C, h*w]")
            tr = ctx.only_consumer(rs.outputs[0], "Transpose")
            if tr is None or tr.attrs.get("perm") != [0, 2, 1]:
                raise RewriteRejected("flattened patches are not transposed to tokens")
            old, out, pos = [cv, rs, tr], tr.outputs[0], None
            ad = ctx.only_consumer(out, "Add")
            pn = ctx.other_input(ad, out) if ad is not None else None
            if pn is not None and g.const(pn) is not None and g.const(pn).numel() == h * w * N:
                pos, out = pn, ad.outputs[0]
                old.append(ad)
            bias = g.consts[cv.inputs[2]].float() if len(cv.inputs) > 2 and cv.inputs[2] else None
            bname = g.add_const("pe_b", bias) if bias is not None else None
            posn = g.add_const("pe_pos", g.consts[pos].float().reshape(h * w, N)) if pos else None
            y = g.fresh("pe_tok")
            y2 = g.fresh("pe_out")
            new = []
            wm = W.reshape(N, -1).float()
            if dt == torch.float32:  # the raw fp32 image (the op splits it into bf16 planes)
                from ..ops.spectral import split_bf16
                ws = g.add_const("pe_ws", split_bf16(wm))
                new.append(amd_node(g, "patch_linear3", [x, ws, bname, posn], [y], p=p))
            else:
                wb = g.add_const("pe_w", wm.to(torch.bfloat16))
                new.append(amd_node(g, "patch_linear", [x, wb, bname, posn], [y], p=p))
            shp = g.add_const("pe_shape", torch.tensor(g.shape(out), dtype=torch.int64))
            new.append(Node("Reshape", "", [y, shp], [y2], {}, g.fresh("pe_reshape")))
            g.meta[y] = ([B * h * w, N], dt)
            g.meta[y2] = (g.shape(out), g.dtype(out))
            err = _verify(ctx, old, new, [x], [out], [y2], _precision_tol(dt))
            ctx.replace(old, new, {out: y2})
            ctx.report.applied.append({"pattern": "patch_embed", "at": cv.name, "rel_l2": err})
        except Exception as e:  # noqa: BLE001 -- any failure keeps the original nodes
            ctx.report.rejected.append({"pattern": "patch_embed", "at": cv.name, "why": _why(e)})


def rewrite_unpatch_head(ctx: Ctx) -> None:
    """MatMul(t [B, h, w, C], W [C, p*p*Co]) -> Reshape [B, h, w, p, p, Co] ->
    Transpose(0, 5, 1, 3, 2, 4) -> Reshape [B, Co, h*p, w*p] -> linear_unpatch(3)."""
    g = ctx.g
    for mm in [n for n in g.nodes if n.is_("MatMul")]:
        if mm not in g.nodes:
            continue
        t, wname = mm.inputs
        W = g.const(wname)
        if W is None or W.dim() != 2 or g.shape(t) is None or len(g.shape(t)) != 4:
            continue
        rs1 = ctx.only_consumer(mm.outputs[0], "Reshape")
        if rs1 is None or len(g.shape(rs1.outputs[0])) != 6:
            continue
        try:
            B, h, w, C = g.shape(t)
            _, _, _, p, p2, Co = g.shape(rs1.outputs[0])
            tr = ctx.only_consumer(rs1.outputs[0], "Transpose")
            if p != p2 or tr is None or tr.attrs.get("perm") != [0, 5, 1, 3, 2, 4]:
                raise RewriteRejected("not the (p1, p2, c_out) un-patchify layout")
            rs2 = ctx.only_consumer(tr.outputs[0], "Reshape")
            if rs2 is None or g.shape(rs2.outputs[0]) != [B, Co, h * p, w * p]:
                raise RewriteRejected("un-patchify does not end in [B, C, h*p, w*p]")
            dt = g.dtype(t)
            if dt not in (torch.float32, torch.bfloat16) or p != 8 or C % 64:
                raise RewriteRejected("head GEMM tile constraints")
            out = rs2.outputs[0]
            # weight rows reordered from (p1, p2, c_out) to (c_out, p1, p2)
            wcpp = W.t().reshape(p, p, Co, C).permute(2, 0, 1, 3).reshape(Co * p * p, C).contiguous().float()
            y = g.fresh("head_out")
            new = []
            if dt == torch.float32:
                from ..ops.spectral import split_bf16
                ts = g.fresh("head_ts")
                new.append(amd_node(g, "split_bf16", [t], [ts], rows=True))
                g.meta[ts] = ([B, h, w, 2 * C], torch.bfloat16)
                ws = g.add_const("head_ws", split_bf16(wcpp))
                g.orig[ws] = wcpp
                new.append(amd_node(g, "linear_unpatch3", [ts, ws, None], [y], C=Co, h=h, w=w, p=p))
            else:
                wb = g.add_const("head_w", wcpp.to(torch.bfloat16))
                new.append(amd_node(g, "linear_unpatch", [t, wb, None], [y], C=Co, h=h, w=w, p=p))
            g.meta[y] = (g.shape(out), g.dtype(out))
            old = [mm, rs1, tr, rs2]
            err = _verify(ctx, old, new, [t], [out], [y], _precision_tol(dt))
            ctx.replace(old, new, {out: y})
            ctx.report.applied.append({"pattern": "unpatch_head", "at": mm.name, "rel_l2": err})
        except Exception as e:  # noqa: BLE001 -- any failure keeps the original nodes
            ctx.report.rejected.append({"pattern": "unpatch_head", "at": mm.name, "why": _why(e)})


# ----------------------------------------------------------------------------------------- spectral regions
@dataclass
class SpectralRegion:
    rfft: Node
    irfft: Node
    nodes: List[Node]  # between rfft and irfft (exclusive)


def _region(ctx: Ctx, rf: Node) -> Optional[SpectralRegion]:
    """Nodes on the paths from ``rf``'s output to exactly one Irfft; every other input of those
    nodes must be a constant and none of their values may escape the region."""
    g = ctx.g
    seen: Dict[int, Node] = {}
    stack = [rf.outputs[0]]
    irffts: Dict[int, Node] = {}
    while stack:
        v = stack.pop()
        for c in ctx.cons.get(v, []):
            if c.is_("Irfft", CONTRIB_DOMAIN):
                irffts[id(c)] = c
                continue
            if id(c) in seen:
                continue
            seen[id(c)] = c
            stack.extend(o for o in c.outputs if o)
    if len(irffts) != 1:
        return None
    ir = next(iter(irffts.values()))
    inside = {rf.outputs[0]} | {o for n in seen.values() for o in n.outputs if o}
    order = [n for n in g.nodes if id(n) in seen]
    for n in order:
        for i in n.inputs:
            if i and i not in inside and i not in g.consts:
                return None
        for o in n.outputs:
            if o in g.output_names:
                return None
            for c in ctx.cons.get(o, []):
                if id(c) not in seen and c is not ir:
                    return None
    if ir.inputs[0] not in inside:
        return None
    return SpectralRegion(rf, ir, order)


def _region_fn(ctx: Ctx, reg: SpectralRegion):
    g = ctx.g

    def F(X: torch.Tensor) -> torch.Tensor:
        env = g.run_nodes(reg.nodes, {reg.rfft.outputs[0]: X}, ctx.device)
        return env[reg.irfft.inputs[0]]

    return F


def _post_chain(ctx: Ctx, v: str, perm: Optional[List[int]]) -> Tuple[List[Node], str, float, bool]:
    """Follow scalar Mul / Div, Casts and (at most one) Transpose(``perm``) from ``v``.
    Returns (nodes, value, scale, transposed)."""
    g = ctx.g
    nodes, scale, transposed = [], 1.0, False
    while True:
        c = ctx.only_consumer(v)
        if c is None:
            break
        if c.is_("Mul") or (c.is_("Div") and c.inputs[0] == v):
            s = g.scalar(ctx.other_input(c, v) or "")
            if s is None:
                break
            scale *= s if c.is_("Mul") else 1.0 / s
        elif c.is_("Transpose") and perm is not None and not transposed and c.attrs.get("perm") == perm:
            transposed = True
        elif c.is_("Cast"):
            pass
        else:
            break
        nodes.append(c)
        v = c.outputs[0]
    return nodes, v, scale, transposed


def _pre_transpose(ctx: Ctx, v: str, perm: List[int]) -> Tuple[List[Node], str, float]:
    """Walk back from ``v`` over scalar Muls, Casts and one Transpose(``perm``):
    (nodes, source, scale)."""
    g = ctx.g
    nodes, scale, seen_t = [], 1.0, False
    while True:
        p = ctx.producer(v)
        if p is None or ctx.only_consumer(v) is None:
            break
        if p.is_("Mul"):
            a, b = p.inputs
            s = g.scalar(b) if g.scalar(b) is not None else g.scalar(a)
            if s is None:
                break
            scale *= s
            v = a if g.scalar(b) is not None else b
        elif p.is_("Transpose") and not seen_t and p.attrs.get("perm") == perm:
            seen_t = True
            v = p.inputs[0]
        elif p.is_("Cast") and P.onnx_dtype_to_torch(p.attrs["to"]) == torch.float32:
            v = p.inputs[0]
        else:
            break
        nodes.append(p)
    # the chain must start at a value with other uses or a non-chain producer (h), not mid-cast
    return (nodes, v, scale) if seen_t else ([], "", 1.0)


def _scalar_consts(ctx: Ctx, nodes: Sequence[Node]) -> List[float]:
    vals = set()
    for n in nodes:
        for i in n.inputs:
            s = ctx.g.scalar(i)
            if s is not None and s != 0.0 and math.isfinite(s):
                vals.add(abs(float(s)))
    return sorted(vals)


def _relu_depth(ctx: Ctx, reg: SpectralRegion) -> Dict[str, int]:
    d = {reg.rfft.outputs[0]: 0}
    for n in reg.nodes:
        k = max([d.get(i, 0) for i in n.inputs if i] + [0]) + (1 if n.is_("Relu") else 0)
        for o in n.outputs:
            d[o] = k
    return d


def rewrite_afno(ctx: Ctx) -> None:
    """The AFNO filter: channel-last Transpose -> Rfft -> block MLP region -> Irfft -> Transpose
    (+ filter input) (+ residual) -> r2c + afno_spectral + c2r_add."""
    from ..models.afno import kept_window  # noqa: F401  (documentation of the window convention)
    from ..ops.spectral import AFNO_FUSED_SHAPES, pack_afno_weights

    g = ctx.g
    for rf in [n for n in g.nodes if n.is_("Rfft", CONTRIB_DOMAIN)]:
        if rf not in g.nodes or rf.attrs.get("signal_ndim", 1) != 2:
            continue
        try:
            pre, h, s_pre = _pre_transpose(ctx, rf.inputs[0], [0, 3, 1, 2])
            if not h:
                continue  # not channel-last: the FNO rewrite may take it
            reg = _region(ctx, rf)
            if reg is None:
                raise RewriteRejected("Rfft ... Irfft is not a closed constant-weight region")
            if reg.irfft.attrs.get("signal_ndim", 1) != 2:
                raise RewriteRejected("Irfft signal_ndim != 2")
            post, y, s_post, tr = _post_chain(ctx, reg.irfft.outputs[0], [0, 2, 3, 1])
            if not tr:
                raise RewriteRejected("Irfft output is not permuted back to channel-last")
            B, H, W, C = g.shape(h)
            dt = g.dtype(h)
            # --- the constants of the block MLP, split into layers by the ReLU depth of their data
            depth = _relu_depth(ctx, reg)
            mats = {0: [], 1: []}
            biases = {0: [], 1: []}
            for n in reg.nodes:
                for i in n.inputs:
                    c = g.const(i)
                    if c is None or not c.is_floating_point() or c.dim() < 2:
                        continue
                    data = [j for j in n.inputs if j and j != i and g.const(j) is None]
                    if not data:
                        continue
                    lay = depth.get(data[0], 0)
                    if lay not in mats:
                        raise RewriteRejected("more than two MLP layers")
                    if c.dim() == 3 and c.shape[1] == c.shape[2]:
                        mats[lay].append(i)
                    elif c.dim() == 2:
                        biases[lay].append(i)
            if any(len(set(mats[k])) != 2 or len(set(biases[k])) != 2 for k in (0, 1)):
                raise RewriteRejected("region is not a two-layer block-diagonal complex MLP")
            mats = {k: sorted(set(v)) for k, v in mats.items()}
            biases = {k: sorted(set(v)) for k, v in biases.items()}
            nb, bs, _ = g.consts[mats[0][0]].shape
            if nb * bs != C:
                raise RewriteRejected("block sizes do not tile the channels")
            F = _region_fn(ctx, reg)
            # --- probe on a realistic spectrum: Rfft of a random channel-last field
            gen = _gen(ctx.device, 7)
            hp = torch.randn([B, H, W, C], generator=gen, device=ctx.device).to(dt)
            pre_env = g.run_nodes(pre[::-1] + [rf], {h: hp}, ctx.device)
            X = pre_env[rf.outputs[0]]
            Y = F(X)
            Yc = Y.float()
            nz = Yc.abs().amax(dim=(0, 1, 4)) > 0  # [H, wf] modes that carry output
            rows = torch.nonzero(nz.any(1)).flatten().tolist()
            cols = torch.nonzero(nz.any(0)).flatten().tolist()
            if not rows or not cols:
                raise RewriteRejected("region output is identically zero")
            r0, r1, km = rows[0], rows[-1] + 1, cols[-1] + 1
            if cols != list(range(km)) or rows != list(range(r0, r1)):
                raise RewriteRejected("kept-mode window is not a leading W range x a contiguous H range")
            if r0 != 0 or r1 != H:
                raise RewriteRejected(f"AFNO window rows {r0}:{r1} (the fused kernel keeps all {H} rows)")
            if (H, bs) not in AFNO_FUSED_SHAPES:
                raise RewriteRejected(f"no fused AFNO kernel for H={H}, block size {bs}")
            # --- roles: which constant is w_re / w_im / b_re / b_im of each layer, the input scale
            # and the softshrink threshold: checked on sampled modes of the probe
            scal = _scalar_consts(ctx, reg.nodes)
            sel = torch.randint(0, B * (r1 - r0) * km, (8,), generator=_gen("cpu", 8))
            Xs = X.float().permute(0, 2, 3, 1, 4)[:, r0:r1, :km].reshape(-1, C, 2)[sel.to(X.device)].cpu().double()
            Ys = Yc.permute(0, 2, 3, 1, 4)[:, r0:r1, :km].reshape(-1, C, 2)[sel.to(Y.device)].cpu().double()
            best = None
            for (w1r, w1i), (b1r, b1i), (w2r, w2i), (b2r, b2i), s_in, s_out, lam in itertools.product(
                    itertools.permutations(mats[0]), itertools.permutations(biases[0]),
                    itertools.permutations(mats[1]), itertools.permutations(biases[1]),
                    [1.0] + scal, [1.0] + scal, [0.0] + scal):
                cw = [g.consts[k].double() for k in (w1r, w1i, w2r, w2i)]
                cb = [g.consts[k].double() for k in (b1r, b1i, b2r, b2i)]
                z = _afno_mlp_ref(Xs * s_in, cw, cb, lam, nb, bs) * s_out
                err = float((z - Ys).norm() / Ys.norm().clamp_min(1e-30))
                if best is None or err < best[0]:
                    best = (err, (w1r, w1i, b1r, b1i, w2r, w2i, b2r, b2i), s_in, s_out, lam)
                if err < 1e-6:
                    break
            if best is None or best[0] > 1e-4:
                raise RewriteRejected(f"region is not the AFNO block MLP (best fit rel {best[0] if best else 'n/a'})")
            _, (w1r, w1i, b1r, b1i, w2r, w2i, b2r, b2i), s_in, s_out, lam = best
            w1 = torch.stack([g.consts[w1r], g.consts[w1i]]).float()
            w2 = torch.stack([g.consts[w2r], g.consts[w2i]]).float()
            b1 = torch.stack([g.consts[b1r], g.consts[b1i]]).float()
            b2 = torch.stack([g.consts[b2r], g.consts[b2i]]).float()
            sdt = torch.float32 if dt == torch.float32 else torch.bfloat16
            w1t, w2t, b1p, b2p = pack_afno_weights(w1, b1, w2, b2, split=sdt == torch.float32)
            # --- skip additions after the filter: + h (the AFNO bias), + residual
            old = pre + [rf] + reg.nodes + [reg.irfft] + post
            out, add1, add2 = y, None, None
            a1 = ctx.only_consumer(out, "Add")
            if a1 is not None and ctx.other_input(a1, out) == h:
                add1, out = h, a1.outputs[0]
                old.append(a1)
                a2 = ctx.only_consumer(out, "Add")
                r = ctx.other_input(a2, out) if a2 is not None else None
                if r is not None and g.shape(r) == [B, H, W, C] and g.dtype(r) == dt and g.const(r) is None:
                    add2, out = r, a2.outputs[0]
                    old.append(a2)
            names = [g.add_const(k, v) for k, v in (("afno_w1t", w1t), ("afno_w2t", w2t), ("afno_b1", b1p),
                                                     ("afno_b2", b2p))]
            xw, yw, o = g.fresh("afno_xw"), g.fresh("afno_yw"), g.fresh("afno_out")
            new = [amd_node(g, "r2c", [h], [xw], dim=[2], scale=float(s_pre * s_in), keep=[km, 0], out_dtype=sdt),
                   amd_node(g, "afno_spectral", [xw] + names, [yw], lam=float(lam)),
                   amd_node(g, "c2r_add", [yw, add1, add2], [o], dim=[2], out_size=[W],
                            scale=float(s_out * s_post / (H * W)), keep=[km, 0], out_dtype=dt)]
            g.meta[xw] = ([B, H, km, C, 2], sdt)
            g.meta[yw] = ([B, H, km, C, 2], sdt)
            g.meta[o] = (g.shape(out), g.dtype(out))
            ins = [h] + ([add2] if add2 else [])
            err = _verify(ctx, old, new, ins, [out], [o], 2e-4 if dt == torch.float32 else 4e-2, scales=(1.0, 4.0))
            ctx.replace(old, new, {out: o})
            ctx.report.applied.append({"pattern": "afno_filter", "at": rf.name, "rel_l2": err, "modes": [r1 - r0, km],
                                       "lambda": lam, "skips": int(add1 is not None) + int(add2 is not None)})
        except Exception as e:  # noqa: BLE001 -- any failure keeps the original nodes
            ctx.report.rejected.append({"pattern": "afno_filter", "at": rf.name, "why": _why(e)})


def _afno_mlp_ref(X: torch.Tensor, w: List[torch.Tensor], b: List[torch.Tensor], lam: float, nb: int, bs: int):
    """Block MLP on sampled modes X [S, C, 2] (float64): FourCastNet's AFNO2D formulas."""
    S = X.shape[0]
    xr, xi = X[..., 0].reshape(S, nb, bs), X[..., 1].reshape(S, nb, bs)
    e = lambda a, m: torch.einsum("sbi,bio->sbo", a, m)  # noqa: E731
    o1r = torch.relu(e(xr, w[0]) - e(xi, w[1]) + b[0])
    o1i = torch.relu(e(xi, w[0]) + e(xr, w[1]) + b[1])
    o2r = e(o1r, w[2]) - e(o1i, w[3]) + b[2]
    o2i = e(o1i, w[2]) + e(o1r, w[3]) + b[3]
    o = torch.stack([o2r, o2i], -1).reshape(S, nb * bs, 2)
    if lam > 0:
        o = torch.where(o > lam, o - lam, torch.where(o < -lam, o + lam, torch.zeros_like(o)))
    return o


def rewrite_fno(ctx: Ctx) -> None:
    """FNO spectral conv: Rfft over the last two dims -> per-mode linear channel mixing on the
    modes [0, m1) u [H - m1, H) x [0, m2) -> Irfft (+ Conv1x1(x) + GELU) -> dftw_r2c + c2c_axis +
    fno_mix_c2c + fno_c2r_pw (without the pointwise branch: fno_c2r, or c2r for other dtypes)."""
    g = ctx.g
    for rf in [n for n in g.nodes if n.is_("Rfft", CONTRIB_DOMAIN)]:
        if rf not in g.nodes or rf.attrs.get("signal_ndim", 1) != 2:
            continue
        try:
            x = rf.inputs[0]
            cast = ctx.producer(x, "Cast")
            pre = []
            if cast is not None and ctx.only_consumer(x) is rf:
                pre, x = [cast], cast.inputs[0]
            if g.shape(x) is None or len(g.shape(x)) != 4:
                continue
            B, Cin, H, W = g.shape(x)
            wf = W // 2 + 1
            reg = _region(ctx, rf)
            if reg is None:
                raise RewriteRejected("Rfft ... Irfft is not a closed constant-weight region")
            if any(n.is_("Relu") or n.is_("Where") for n in reg.nodes):
                continue  # non-linear region (AFNO-like)
            F = _region_fn(ctx, reg)
            ysh = g.shape(reg.irfft.inputs[0])
            if ysh is None or len(ysh) != 5 or ysh[0] != B or ysh[2:] != [H, wf, 2]:
                raise RewriteRejected("mixing does not keep the [B, C, H, W/2+1, 2] layout")
            Cout = ysh[1]
            dev = ctx.device
            # --- per-mode weights from unit probes (one input channel per batch row)
            Wt = torch.zeros(Cin, Cout, H, wf, 2, dtype=torch.float64)
            for c0 in range(0, Cin, B):
                X = torch.zeros(B, Cin, H, wf, 2, device=dev)
                for b in range(min(B, Cin - c0)):
                    X[b, c0 + b, :, :, 0] = 1.0
                Y = F(X).double().cpu()
                for b in range(min(B, Cin - c0)):
                    Wt[c0 + b] = Y[b]
            nzm = (Wt.abs().amax(dim=(0, 1, 4)) > 0)
            rows = torch.nonzero(nzm.any(1)).flatten().tolist()
            cols = torch.nonzero(nzm.any(0)).flatten().tolist()
            if not rows or not cols:
                raise RewriteRejected("mixing is identically zero")
            m2 = cols[-1] + 1
            lo = [r for r in rows if r < H // 2]
            m1 = (lo[-1] + 1) if lo else 0
            if cols != list(range(m2)) or m1 == 0 or rows != list(range(m1)) + list(range(H - m1, H)):
                raise RewriteRejected("mode window is not [0, m1) u [H-m1, H) x [0, m2)")
            keep_rows = list(range(m1)) + list(range(H - m1, H))
            Wk = Wt[:, :, keep_rows, :m2]  # [Cin, Cout, 2*m1, m2, 2] (complex-as-pair)
            # --- the map must be complex-linear, batch- and mode-diagonal: check on random spectra
            gen = _gen("cpu", 11)
            Xr = torch.randn(B, Cin, H, wf, 2, generator=gen, dtype=torch.float64)
            Yr = F(Xr.float().to(dev)).double().cpu()
            wc = torch.view_as_complex(Wk.contiguous())
            xc = torch.view_as_complex(Xr[:, :, keep_rows, :m2].contiguous())
            pred = torch.zeros(B, Cout, H, wf, dtype=torch.complex128)
            pred[:, :, keep_rows, :m2] = torch.einsum("bixy,ioxy->boxy", xc, wc)
            if _rel(torch.view_as_real(pred), Yr) > 1e-5:
                raise RewriteRejected("region is not a per-mode complex-linear channel mixing")
            post, y, s_post, _ = _post_chain(ctx, reg.irfft.outputs[0], None)
            dt = g.dtype(y)
            old = pre + [rf] + reg.nodes + [reg.irfft] + post
            out = y
            # (+ Conv1x1(x) + bias) (+ GELU): the FNO layer's pointwise branch
            conv, gelu = None, False
            ad = ctx.only_consumer(out, "Add")
            cvn = ctx.producer(ctx.other_input(ad, out) or "", "Conv") if ad is not None else None
            if cvn is not None and cvn.inputs[0] == x and ctx.only_consumer(cvn.outputs[0]) is ad:
                Wc = g.const(cvn.inputs[1])
                if Wc is not None and tuple(Wc.shape) == (Cout, Cin, 1, 1) and cvn.attrs.get("group", 1) == 1 and \
                        not any(cvn.attrs.get("pads", [0] * 4)) and all(s == 1 for s in cvn.attrs.get("strides", [1, 1])):
                    conv = cvn
                    old += [cvn, ad]
                    out = ad.outputs[0]
                    ge = _gelu_after(ctx, out)
                    if ge is not None:
                        old += ge[0]
                        out, gelu = ge[1], True
            wpk = g.add_const("fno_w", Wk.reshape(Cin, Cout, 2 * m1 * m2, 2).float())
            xw, xm, yw, o = g.fresh("fno_xw"), g.fresh("fno_xm"), g.fresh("fno_yw"), g.fresh("fno_out")
            new = [amd_node(g, "dftw_r2c", [x], [xw], m=m2, scale=1.0),
                   amd_node(g, "c2c_axis", [xw], [xm], dim=2, n=H, in_lo=H, in_hi=0, out_lo=m1, out_hi=m1,
                            inverse=False, scale=1.0),
                   amd_node(g, "fno_mix_c2c", [xm, wpk], [yw], n=H, in_lo=m1, in_hi=m1,
                            scale=float(s_post / (H * W)), path=0)]
            g.meta[xw] = ([B, Cin, H, m2, 2], torch.float32)
            g.meta[xm] = ([B, Cin, 2 * m1, m2, 2], torch.float32)
            g.meta[yw] = ([B, Cout, H, m2, 2], torch.float32)
            if conv is not None:
                wcn = g.add_const("fno_pw_w", g.consts[conv.inputs[1]].reshape(Cout, Cin).float())
                bcn = g.add_const("fno_pw_b", g.consts[conv.inputs[2]].float()) if len(conv.inputs) > 2 and \
                    conv.inputs[2] else None
                new.append(amd_node(g, "fno_c2r_pw", [yw, x, wcn, bcn], [o], gelu=gelu))
            elif dt in (torch.float32, torch.bfloat16):  # SpectralConv2d alone: the layer tail without x
                new.append(amd_node(g, "fno_c2r", [yw], [o], W=W, out_dtype=dt))
            else:
                new.append(amd_node(g, "c2r", [yw], [o], dim=[3], out_size=[W], scale=1.0, keep=[m2, 0], out_dtype=dt))
            g.meta[o] = (g.shape(out), g.dtype(out))
            err = _verify(ctx, old, new, [x], [out], [o], 2e-4 if dt == torch.float32 else 4e-2)
            ctx.replace(old, new, {out: o})
            ctx.report.applied.append({"pattern": "fno_spectral" + ("_pointwise" if conv is not None else "")
                                       + ("_gelu" if gelu else ""), "at": rf.name, "rel_l2": err, "modes": [m1, m2]})
        except Exception as e:  # noqa: BLE001 -- any failure keeps the original nodes
            ctx.report.rejected.append({"pattern": "fno_spectral", "at": rf.name, "why": _why(e)})


# ----------------------------------------------------------------------------------------- whole blocks
def _amd(n: Optional[Node], op: str) -> bool:
    return n is not None and n.domain == AMD_DOMAIN and n.op == op


def _mask(n: Node) -> List[int]:
    return list(n.attrs.get("tensor_mask", []))


def _users(ctx: Ctx, v: str) -> List[Node]:
    return [] if v in ctx.g.output_names else ctx.cons.get(v, [])


def _weight_f32(g: IRGraph, ws: str) -> torch.Tensor:
    """fp32 [N, K] weight behind a split-pair constant (the original when a rewrite recorded it)."""
    if ws in g.orig:
        return g.orig[ws].float()
    from ..ops.spectral import unsplit_bf16
    return unsplit_bf16(g.consts[ws]).float()


def _block_nodes(ctx: Ctx, c2r: Node):
    """The fp32 FourCastNet block around an AFNO ``c2r_add`` as the earlier passes leave it:
    h = layer_norm(x); xw = r2c(h); yw = afno_spectral(xw); x1 = c2r_add(yw, h, x);
    x1s = layer_norm_split(x1); hid = linear3(x1s, GELU, split out); y = linear3(hid, + b2, + x1).
    Returns the nodes or None."""
    g = ctx.g
    if _mask(c2r)[:3] != [1, 1, 1] or c2r.attrs.get("out_dtype") != _SCALARTYPE[torch.float32]:
        return None
    yw, h, x = c2r.inputs[:3]
    ln1, sp = ctx.producer(h), ctx.producer(yw)
    if not _amd(ln1, "layer_norm") or ln1.outputs[0] != h or ln1.inputs[0] != x or _mask(ln1) != [1, 1, 1, 0] \
            or _users(ctx, ln1.outputs[1]) or not _amd(sp, "afno_spectral") or _users(ctx, yw) != [c2r]:
        return None
    r2c = ctx.producer(sp.inputs[0])
    if not _amd(r2c, "r2c") or r2c.inputs[0] != h or r2c.attrs.get("dim") != [2] or \
            _users(ctx, sp.inputs[0]) != [sp] or sorted(map(id, _users(ctx, h))) != sorted([id(r2c), id(c2r)]):
        return None
    if r2c.attrs.get("out_dtype") != _SCALARTYPE[torch.float32] or g.dtype(x) != torch.float32 or \
            len(g.shape(x) or []) != 4:
        return None
    x1 = c2r.outputs[0]
    us = _users(ctx, x1)
    lns = next((u for u in us if _amd(u, "layer_norm_split")), None)
    if lns is None or len(us) != 2 or lns.inputs[0] != x1 or _mask(lns) != [1, 1, 1, 0]:
        return None
    fc1 = ctx.only_consumer(lns.outputs[0])
    if not _amd(fc1, "linear3") or _mask(fc1) != [1, 1, 1, 0] or fc1.attrs.get("act") != 1 or \
            not fc1.attrs.get("split_out"):
        return None
    fc2 = ctx.only_consumer(fc1.outputs[0])
    if not _amd(fc2, "linear3") or fc2 not in us or _mask(fc2) != [1, 1, 1, 1] or fc2.inputs[3] != x1 or \
            fc2.attrs.get("act", 0) != 0 or fc2.attrs.get("split_out"):
        return None
    return ln1, r2c, sp, c2r, lns, fc1, fc2


def fuse_afno_blocks(ctx: Ctx) -> None:
    """fp32 FourCastNet blocks -> the native block sequence (ops/spectral.py afno_block_fused_f32):
    LN1 applied inside the W-transform's loads (``r2c_ln``; the normalised copy of x is never
    stored), the C2R epilogue adding both skips, writing fc1's centred split pairs and LN2's
    partial statistics (``c2r_ln_add_split``), and LN2 folded into fc1's epilogue (``linear3_ln``):
    two full-tensor passes fewer per block.  Then, across blocks, fc2 emits the next block's LN1
    partial statistics (``linear3_stats``) with its bias carried as the next block's ``pre``, and
    the last fc2 writes the head's split pairs itself with its bias folded into the head's."""
    from ..ops.spectral import split_bf16, unsplit_bf16

    g = ctx.g
    for c2r in [n for n in g.nodes if _amd(n, "c2r_add")]:
        blk = _block_nodes(ctx, c2r)
        if blk is None:
            continue
        ln1, r2c, sp, c2r, lns, fc1, fc2 = blk
        try:
            x, g1, b1 = ln1.inputs[:3]
            g2, b2 = lns.inputs[1:3]
            B, H, W, C = g.shape(x)
            if C % 64 or C > 64 * 64:
                raise RewriteRejected("LN partial statistics need C % 64 == 0 and C <= 4096")
            km = r2c.attrs["keep"][0]
            w1 = _weight_f32(g, fc1.inputs[1]).double()
            gam, bet = g.consts[g2].double().reshape(C), g.consts[b2].double().reshape(C)
            w1s = split_bf16((w1 * gam[None, :]).float())
            c1 = unsplit_bf16(w1s).double().sum(1).float()
            c2 = (w1 @ bet + g.consts[fc1.inputs[2]].double()).float()
            n_w1s, n_c1, n_c2 = g.add_const("blk_w1s", w1s), g.add_const("blk_c1", c1), g.add_const("blk_c2", c2)
            st, xw, yw = g.fresh("blk_st"), g.fresh("blk_xw"), g.fresh("blk_yw")
            x1, x1s2, part2 = g.fresh("blk_x1"), g.fresh("blk_x1s2d"), g.fresh("blk_part2")
            x1s, st2, hid, y = g.fresh("blk_x1s"), g.fresh("blk_st2"), g.fresh("blk_hid"), g.fresh("blk_y")
            shp = g.add_const("blk_shape", torch.tensor([B, H, W, 2 * C], dtype=torch.int64))
            new = [amd_node(g, "ln_stats", [x, None], [st], eps=ln1.attrs["eps"]),
                   amd_node(g, "r2c_ln", [x, st, g1, b1, None], [xw], dim=2, scale=r2c.attrs["scale"], keep=km,
                            out_dtype=torch.float32),
                   Node(sp.op, sp.domain, [xw] + sp.inputs[1:], [yw], dict(sp.attrs), g.fresh("afno_spectral")),
                   amd_node(g, "c2r_ln_add_split", [yw, x, st, g1, b1, None], [x1, x1s2, part2], dim=2, n=W,
                            scale=c2r.attrs["scale"]),
                   Node("Reshape", "", [x1s2, shp], [x1s], {}, g.fresh("reshape")),
                   amd_node(g, "ln_stats_merge", [part2, st], [st2], eps=lns.attrs["eps"]),
                   amd_node(g, "linear3_ln", [x1s, n_w1s, n_c1, n_c2, st2], [hid], act=1),
                   Node(fc2.op, fc2.domain, [hid, fc2.inputs[1], fc2.inputs[2], x1], [y], dict(fc2.attrs),
                        g.fresh("linear3"))]
            M = B * H * W
            for k, v in ((st, ([M, 2], torch.float32)), (xw, (g.shape(sp.inputs[0]), torch.float32)),
                         (yw, (g.shape(sp.inputs[0]), torch.float32)), (x1, ([B, H, W, C], torch.float32)),
                         (x1s2, ([M, 2 * C], torch.bfloat16)), (part2, ([M, C // 64, 2], torch.float32)),
                         (x1s, ([B, H, W, 2 * C], torch.bfloat16)), (st2, ([M, 2], torch.float32)),
                         (hid, (g.shape(fc1.outputs[0]), torch.bfloat16)), (y, g.meta[fc2.outputs[0]])):
                g.meta[k] = v
            old = list(blk)
            err = _verify(ctx, old, new, [x], [fc2.outputs[0]], [y], 2e-4, scales=(1.0, 4.0))
            ctx.replace(old, new, {fc2.outputs[0]: y})
            ctx.report.applied.append({"pattern": "afno_block", "at": c2r.name, "rel_l2": err})
        except Exception as e:  # noqa: BLE001 -- any failure keeps the original nodes
            ctx.report.rejected.append({"pattern": "afno_block", "at": c2r.name, "why": _why(e)})
    _chain_afno_blocks(ctx)


def _chain_afno_blocks(ctx: Ctx) -> None:
    from ..ops.spectral import split_bf16

    g = ctx.g
    for fc2 in [n for n in g.nodes if _amd(n, "linear3")]:
        if fc2 not in g.nodes or _mask(fc2) != [1, 1, 1, 1] or fc2.attrs.get("act", 0) or fc2.attrs.get("split_out"):
            continue
        hid, w2s, b2, res = fc2.inputs
        v = fc2.outputs[0]
        us = _users(ctx, v)
        try:
            st = next((u for u in us if _amd(u, "ln_stats")), None)
            r2 = next((u for u in us if _amd(u, "r2c_ln")), None)
            cs = next((u for u in us if _amd(u, "c2r_ln_add_split")), None)
            if st is not None and r2 is not None and cs is not None and len(us) == 3 and \
                    _mask(st) == [1, 0] and _mask(r2)[4] == 0 and _mask(cs)[5] == 0:
                # fc2 -> next block: statistics from fc2's epilogue, bias carried as `pre`
                sp = ctx.producer(cs.inputs[0])
                C = g.shape(v)[-1]
                M = math.prod(g.shape(v)) // C
                y, part, stn = g.fresh("blk_y"), g.fresh("blk_part"), g.fresh("blk_st")
                xw, yw = g.fresh("blk_xw"), g.fresh("blk_yw")
                outs_cs = [g.fresh("blk_x1"), g.fresh("blk_x1s2d"), g.fresh("blk_part2")]
                new = [amd_node(g, "linear3_stats", [hid, w2s, res, b2], [y, part]),
                       amd_node(g, "ln_stats_merge", [part, None], [stn], eps=st.attrs["eps"]),
                       amd_node(g, "r2c_ln", [y, stn] + r2.inputs[2:4] + [b2], [xw], dim=r2.attrs["dim"],
                                scale=r2.attrs["scale"], keep=r2.attrs["keep"], out_dtype=torch.float32),
                       Node(sp.op, sp.domain, [xw] + sp.inputs[1:], [yw], dict(sp.attrs), g.fresh("afno_spectral")),
                       amd_node(g, "c2r_ln_add_split", [yw, y, stn] + cs.inputs[3:5] + [b2], outs_cs,
                                dim=cs.attrs["dim"], n=cs.attrs["n"], scale=cs.attrs["scale"])]
                for k, m in ((y, g.meta[v]), (part, ([M, C // 64, 2], torch.float32)), (stn, ([M, 2], torch.float32)),
                             (xw, g.meta[r2.outputs[0]]), (yw, g.meta[sp.outputs[0]])):
                    g.meta[k] = m
                for a, b in zip(cs.outputs, outs_cs):
                    g.meta[b] = g.meta[a]
                old = [fc2, st, r2, sp, cs]
                err = _verify(ctx, old, new, [hid, res], cs.outputs, outs_cs, 2e-4)
                ctx.replace(old, new, dict(zip(cs.outputs, outs_cs), **{st.outputs[0]: stn}))
                ctx.report.applied.append({"pattern": "afno_block_chain", "at": fc2.name, "rel_l2": err})
                continue
            sp_ = us[0] if len(us) == 1 and _amd(us[0], "split_bf16") and us[0].attrs.get("rows", True) else None
            head = ctx.only_consumer(sp_.outputs[0]) if sp_ is not None else None
            if _amd(head, "linear_unpatch3"):
                # last fc2 -> head: split pairs straight from fc2, its bias folded into the head's
                hws = head.inputs[1]
                hb = g.consts[head.inputs[2]].double() if _mask(head)[2] else 0.0
                bias = (_weight_f32(g, hws).double() @ g.consts[b2].double() + hb).float()
                ys, hy = g.fresh("blk_ys"), g.fresh("head_out")
                new = [amd_node(g, "linear3", [hid, w2s, None, res], [ys], act=0, split_out=True),
                       Node(head.op, head.domain, [ys, hws, g.add_const("head_b", bias)], [hy],
                            dict(head.attrs, tensor_mask=[1, 1, 1]), g.fresh("linear_unpatch3"))]
                g.meta[ys] = g.meta[sp_.outputs[0]]
                g.meta[hy] = g.meta[head.outputs[0]]
                old = [fc2, sp_, head]
                err = _verify(ctx, old, new, [hid, res], [head.outputs[0]], [hy], 2e-4)
                ctx.replace(old, new, {head.outputs[0]: hy})
                ctx.report.applied.append({"pattern": "afno_block_head", "at": fc2.name, "rel_l2": err})
        except Exception as e:  # noqa: BLE001 -- any failure keeps the original nodes
            ctx.report.rejected.append({"pattern": "afno_block_chain", "at": fc2.name, "why": _why(e)})


# ----------------------------------------------------------------------------------------- driver
PASSES = (("afno_filter", rewrite_afno), ("fno_spectral", rewrite_fno), ("layer_norm", rewrite_layernorm),
          ("patch_embed", rewrite_patch_embed), ("unpatch_head", rewrite_unpatch_head), ("linear", rewrite_linear),
          ("pointwise_conv", rewrite_pointwise_conv), ("split_fusion", fuse_split_chains),
          ("afno_block", fuse_afno_blocks))


def optimize(onnx_bytes: bytes, input_shapes: Sequence[Sequence[int]], input_dtypes=None, device=None,
             verify: bool = True, passes: Optional[Sequence[str]] = None, progress=None) -> Tuple[bytes, OptimizeReport]:
    """Rewrite ``onnx_bytes`` for this library's kernels.  Returns (model bytes, report); the
    input bytes are returned unchanged when no rewrite applies.  ``progress(msg)`` is called after
    every pass (engine builds log it)."""
    device = torch.device(device) if device is not None else (
        torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
    model = P.load_model(onnx_bytes)
    g = IRGraph(model, input_shapes, input_dtypes)
    rep = OptimizeReport(nodes_before=len(g.nodes))
    g.fold_constants()
    g.infer_shapes()
    while g.fold_shapes():
        g.fold_constants()
        g.infer_shapes()
    g.eliminate_noops()
    g.dead_code()
    ctx = Ctx(g, device, rep, verify, progress)
    for name, fn in PASSES:
        if passes is not None and name not in passes:
            continue
        n0 = len(rep.applied)
        fn(ctx)
        ctx.topo_fix()
        g.dead_code()
        ctx.refresh()
        if progress is not None:
            progress(f"pass {name}: {len(rep.applied) - n0} rewrites, {len(g.nodes)} nodes")
    rep.nodes_after = len(g.nodes)
    if not rep.applied:
        return onnx_bytes, rep
    return g.to_model().SerializeToString(), rep
