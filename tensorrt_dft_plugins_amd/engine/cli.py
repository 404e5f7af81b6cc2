"""``dftexec``: trtexec-like command line for building, saving, loading and timing engines.

Flag parity with the trtexec invocations of the reference README (README.md:61-75):
``--buildOnly --onnx=... --saveEngine=... --plugins=...`` and ``--loadEngine=... --plugins=...``,
plus ``--shapes`` (README.md:69).  Examples::

    dftexec --buildOnly --onnx=model.onnx --saveEngine=model.engine --plugins=tensorrt_dft_plugins_amd/_C.so
    dftexec --loadEngine=model.engine --plugins=tensorrt_dft_plugins_amd/_C.so --iterations=200
"""
from __future__ import annotations

import argparse
import json
import sys
from typing import List, Optional

import torch


def _parse_shapes(spec: Optional[str]) -> Optional[dict]:
    """``name:1x3x8x8,other:2x4`` -> {name: [1,3,8,8], ...}"""
    if not spec:
        return None
    out = {}
    for part in spec.split(","):
        name, dims = part.rsplit(":", 1)
        out[name.strip("'\"")] = [int(d) for d in dims.split("x")]
    return out


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="dftexec", description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--onnx", help="ONNX model to build an engine from")
    ap.add_argument("--saveEngine", help="write the serialized engine here")
    ap.add_argument("--loadEngine", help="load a serialized engine")
    ap.add_argument("--plugins", action="append", default=[], help="plugin library to load (the op .so)")
    ap.add_argument("--buildOnly", action="store_true", help="build (and save) without running inference")
    ap.add_argument("--shapes", help="static input shapes, e.g. input:1x3x720x1440")
    ap.add_argument("--iterations", type=int, default=100)
    ap.add_argument("--warmUp", type=int, default=10, help="warm-up enqueues before timing")
    ap.add_argument("--noCudaGraph", action="store_true", help="run eagerly instead of replaying a hipGraph")
    ap.add_argument("--device", default=None)
    ap.add_argument("--exportTimes", help="write the timing summary as JSON")
    ap.add_argument("--noOptimize", action="store_true",
                    help="build without the graph rewrite pass (stock nodes run one by one; comparator)")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args(argv)

    if a.verbose:  # engine build / optimizer progress on stderr
        import logging

        from ..utils.trace import get_logger

        get_logger().setLevel(logging.INFO)
    from .. import load_plugins
    from .engine import Engine

    for p in a.plugins:
        from .._loader import native_library_path

        if p and p != native_library_path() and not p.endswith("_C.so"):
            torch.ops.load_library(p)
    load_plugins()
    device = torch.device(a.device) if a.device else None
    if a.loadEngine:
        eng = Engine.load(a.loadEngine, device=device, use_graph=not a.noCudaGraph)
        print(f"[dftexec] loaded engine {a.loadEngine} (arch {eng.header.arch}, format {eng.header.format_version})")
    elif a.onnx:
        shapes = _parse_shapes(a.shapes)
        from .engine import graph_inputs

        ins = graph_inputs(open(a.onnx, "rb").read())
        in_shapes = None
        if shapes is not None:
            in_shapes = [shapes.get(n, s) for n, s, _ in ins]
        eng = Engine.build(a.onnx, shapes=in_shapes, device=device, use_graph=not a.noCudaGraph,
                           optimize=not a.noOptimize)
        print(f"[dftexec] built engine from {a.onnx}")
        opt = eng.header.extra.get("optimizer")
        if opt is not None:
            print(f"[dftexec] graph optimizer: {opt['nodes_before']} -> {opt['nodes_after']} nodes, "
                  f"rewrites {opt['applied']} ({opt['seconds']} s)")
            for r in opt["rejected"] if a.verbose else []:
                print(f"[dftexec]   kept {r['pattern']} at {r['at']}: {r['why']}")
    else:
        ap.error("one of --onnx or --loadEngine is required")
        return 2
    for b in eng.bindings:
        print(f"[dftexec]   {'input ' if b.is_input else 'output'} {b.name}: {b.shape} {b.dtype}")
    if a.saveEngine:
        eng.save(a.saveEngine)
        print(f"[dftexec] saved engine to {a.saveEngine}")
    if a.buildOnly:
        return 0
    stats = eng.benchmark(iterations=a.iterations, warmup=a.warmUp)
    print(f"[dftexec] Throughput: {stats['throughput_qps']:.2f} qps")
    print(f"[dftexec] Latency: min = {stats['latency_min_ms']:.4f} ms, mean = {stats['latency_mean_ms']:.4f} ms, "
          f"median = {stats['latency_median_ms']:.4f} ms, percentile(99%) = {stats['latency_p99_ms']:.4f} ms, "
          f"max = {stats['latency_max_ms']:.4f} ms")
    if a.exportTimes:
        with open(a.exportTimes, "w") as f:
            json.dump(stats, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
