"""In-step marginal cost of each fp32 FourCastNet block stage, without a profiler: the captured
step is timed with one stage run twice per block (MI_DFT_DUP=<stage>, ops/spectral.py), in one
child process per setting; (t_dup - t_base) / depth = that stage's cost inside the real step
(same clocks, caches and neighbours as the benchmark, none of rocprofv3's serialisation).

Usage: python bench/marginal_cost.py [--stages ln_stats,r2c,spectral,c2r,ln_split,fc1,fc2] [--steps 8]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, time, json, torch
sys.path.insert(0, %(root)r)
import tensorrt_dft_plugins_amd as tdp
from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet
from tensorrt_dft_plugins_amd.engine.capture import CapturedModule
tdp.load_plugins()
torch.manual_seed(1234)
cfg = AFNOConfig(depth=%(depth)d)
m = AFNONet(cfg, backend="amd").cuda().eval()
x = torch.randn(%(batch)d, cfg.in_chans, *cfg.img_size, device="cuda")
cap = CapturedModule(m, [x], warmup=2)
for _ in range(3):
    cap.replay()
torch.cuda.synchronize()
ts = []
for _ in range(%(steps)d):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); cap.replay(); e1.record(); torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
ts.sort()
print(json.dumps({"ms": ts[len(ts) // 2], "min": ts[0]}))
"""


def run(stage, a):
    env = dict(os.environ, MI_DFT_DUP=stage)
    code = CHILD % {"root": ROOT, "depth": a.depth, "batch": a.batch, "steps": a.steps}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise SystemExit(f"stage {stage!r} failed:\n{r.stderr[-2000:]}")
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stages", default="ln_stats,r2c,spectral,c2r,ln_split,fc1,fc2")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    base = run("", a)
    print(f"base step: {base['ms']:.2f} ms (min {base['min']:.2f})", flush=True)
    for st in a.stages.split(","):
        r = run(st, a)
        print(f"{st:10s} step {r['ms']:8.2f} ms  marginal per call {(r['ms'] - base['ms']) / a.depth * 1000:8.1f} us"
              f"  (min-based {(r['min'] - base['min']) / a.depth * 1000:8.1f} us)", flush=True)
    base2 = run("", a)
    print(f"base step again: {base2['ms']:.2f} ms (min {base2['min']:.2f})", flush=True)


if __name__ == "__main__":
    main()
