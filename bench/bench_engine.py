"""FourCastNet through the serialized engine (BASELINE config 4 "hipGraph engine"): export the
full model (720x1440, depth 12, batch 32) with its com.amd.dft nodes, Engine.save, Engine.load,
replay; time the loaded engine against the directly captured module (interleaved rounds) and
print dftexec's timing of the same file.

Usage: python bench/bench_engine.py [--dtype fp32|bf16] [--batch 32] [--depth 12] [--out /tmp/fcn.engine]
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from tensorrt_dft_plugins_amd.engine import Engine  # noqa: E402
from tensorrt_dft_plugins_amd.engine.capture import CapturedModule  # noqa: E402
from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet  # noqa: E402


def ms_per(fn, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1000.0 / n


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default="/tmp/fourcastnet.engine")
    a = ap.parse_args(argv)
    tdp.load_plugins()
    dt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    torch.manual_seed(0)
    m = AFNONet(AFNOConfig(depth=a.depth), backend="amd").cuda().to(dt).eval()
    x = torch.randn(a.batch, 20, 720, 1440, device="cuda").to(dt)
    cap = CapturedModule(m, [x])
    t0 = time.perf_counter()
    eng = Engine.build(m, (x,))
    t_build = time.perf_counter() - t0
    eng.save(a.out)
    size = os.path.getsize(a.out)
    del eng
    torch.cuda.empty_cache()
    t0 = time.perf_counter()
    eng = Engine.load(a.out)
    t_load = time.perf_counter() - t0
    (ref,) = cap.replay()
    eng.static_inputs[0].copy_(x)
    eng.enqueue()
    y = eng.static_outputs[0]
    err = float((y.float() - ref.float()).norm() / ref.float().norm())
    res = {"module_ms": [], "engine_ms": []}
    for _ in range(a.rounds):
        res["module_ms"].append(ms_per(cap.replay, a.steps))
        res["engine_ms"].append(ms_per(eng.enqueue, a.steps))
    out = {k: round(statistics.median(v), 3) for k, v in res.items()}
    out.update({"dtype": a.dtype, "batch": a.batch, "depth": a.depth, "engine_bytes": size,
                "build_s": round(t_build, 1), "load_s": round(t_load, 1), "rel_l2_engine_vs_module": err,
                "engine_samples_per_s": round(a.batch * 1000.0 / out["engine_ms"], 2),
                "engine_vs_module": round(out["engine_ms"] / out["module_ms"], 4)})
    print(json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    main()
