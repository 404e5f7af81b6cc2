"""The reference's workflow, timed the reference's way (/root/reference/README.md:57-75):
model -> ONNX file -> ``dftexec --buildOnly --onnx --saveEngine`` -> ``dftexec --loadEngine``.

Three FourCastNet engines (720x1440, depth 12, batch 32, fp32, random init), each built and then
timed from its saved file in a fresh ``dftexec`` process:
  contrib-opt   stock export (OnnxRfft2/OnnxIrfft2 + einsums/LayerNorm/MatMul) with the build-time
                graph rewrite (onnx/optimizer.py) -- the reference workflow on this library
  contrib-raw   the same ONNX file built with --noOptimize (stock nodes one by one; FFTs still on
                the hand kernels)
  amd           the library-native export (com.amd.dft nodes; bench.py's headline engine)
and optionally the contrib FNO2d (BASELINE config 3 layer stack).  Prints one JSON line per engine.

  python bench/bench_contrib.py [--depth 12] [--batch 32] [--iters 20] [--which contrib-opt,contrib-raw,amd,fno]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet, FNO2d, FNOConfig  # noqa: E402
from tensorrt_dft_plugins_amd.onnx import exporter as ex  # noqa: E402


def dftexec(args, timeout=1200):
    """Run the CLI in a fresh process; its stdout is collected and, like its stderr (--verbose
    progress), echoed as it arrives."""
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    t0 = time.time()
    pr = subprocess.Popen([sys.executable, "-m", "tensorrt_dft_plugins_amd.engine.cli", "--verbose"] + args,
                          stdout=subprocess.PIPE, stderr=None, text=True, env=env, cwd=ROOT)
    out = []
    for ln in pr.stdout:
        out.append(ln)
        print(ln.rstrip(), file=sys.stderr, flush=True)
    rc = pr.wait(timeout=timeout)
    if rc != 0:
        raise RuntimeError(f"dftexec {' '.join(args)} failed ({rc})")
    return "".join(out), time.time() - t0


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--which", default="contrib-opt,contrib-raw,amd,fno")
    ap.add_argument("--dir", default=None)
    a = ap.parse_args()
    which = a.which.split(",")
    d = a.dir or tempfile.mkdtemp(prefix="amd_dft_contrib_")
    os.makedirs(d, exist_ok=True)
    cfg = AFNOConfig(depth=a.depth)
    torch.manual_seed(0)
    x = torch.randn(a.batch, cfg.in_chans, *cfg.img_size, device="cuda")
    jobs = []
    if any(w.startswith("contrib") for w in which):
        m = AFNONet(cfg, backend="contrib").cuda().eval()
        path = os.path.join(d, "fourcastnet_contrib.onnx")
        t0 = time.time()
        ex.export(m, (x,), path)
        print(f"[contrib] exported {path} ({os.path.getsize(path) / 1e6:.0f} MB) in {time.time() - t0:.1f}s",
              file=sys.stderr, flush=True)
        del m
        torch.cuda.empty_cache()
        if "contrib-opt" in which:
            jobs.append(("contrib-opt", path, []))
        if "contrib-raw" in which:
            jobs.append(("contrib-raw", path, ["--noOptimize"]))
    if "amd" in which:
        m = AFNONet(cfg, backend="amd").cuda().eval()
        path = os.path.join(d, "fourcastnet_amd.onnx")
        with torch.no_grad():
            ex.export(m, (x,), path)
        del m
        torch.cuda.empty_cache()
        jobs.append(("amd", path, []))
    if "fno" in which:
        fcfg = FNOConfig()
        f = FNO2d(fcfg, backend="contrib").cuda().eval()
        xf = torch.randn(1, fcfg.in_chans, *fcfg.img_size, device="cuda")
        path = os.path.join(d, "fno2d_contrib.onnx")
        ex.export(f, (xf,), path)
        jobs.append(("fno-contrib-opt", path, []))
        jobs.append(("fno-contrib-raw", path, ["--noOptimize"]))
    del x
    torch.cuda.empty_cache()
    for tag, onnx_path, extra in jobs:
        eng = os.path.join(d, tag + ".engine")
        out, tb = dftexec(["--buildOnly", f"--onnx={onnx_path}", f"--saveEngine={eng}",
                           "--plugins=tensorrt_dft_plugins_amd/_C.so"] + extra)
        opt = [ln for ln in out.splitlines() if "graph optimizer" in ln]
        times = os.path.join(d, tag + ".json")
        iters = a.iters if "raw" not in tag else max(3, a.iters // 4)
        out2, tl = dftexec([f"--loadEngine={eng}", "--plugins=tensorrt_dft_plugins_amd/_C.so",
                            f"--iterations={iters}", "--warmUp=3", f"--exportTimes={times}"])
        st = json.load(open(times))
        batch = a.batch if not tag.startswith("fno") else 1
        res = {"engine": tag, "engine_mb": round(os.path.getsize(eng) / 1e6, 1), "build_s": round(tb, 1),
               "load_and_time_s": round(tl, 1), "median_ms": round(st["latency_median_ms"], 3),
               "min_ms": round(st["latency_min_ms"], 3), "iterations": iters,
               "samples_per_s": round(batch / (st["latency_median_ms"] / 1e3), 2), "batch": batch,
               "depth": a.depth if not tag.startswith("fno") else None,
               "optimizer": re.sub(r"^\[dftexec\] graph optimizer: ", "", opt[0]) if opt else None}
        print(json.dumps(res), flush=True)
        os.remove(eng)


if __name__ == "__main__":
    main()
