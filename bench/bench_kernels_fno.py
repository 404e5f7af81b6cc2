"""Per-kernel timing of the FNO layer kernels on the BASELINE config-3 shapes, with variants
that switch parts of the work off (activation, channel counts, modes) to see what bounds them.

Usage: python bench/bench_kernels_fno.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from bench.bench_fft import time_graph  # noqa: E402


def main():
    tdp.load_plugins()
    ops = torch.ops.amd_dft
    dev = "cuda"
    H, W = 720, 1440
    res = {}
    for dt in (torch.bfloat16, torch.float32):
        tag = "bf16" if dt == torch.bfloat16 else "fp32"
        for (B, Ci, Co, m, gelu) in [(1, 20, 20, 32, True), (1, 20, 20, 32, False), (1, 4, 20, 32, True),
                                     (1, 20, 16, 32, True), (1, 20, 20, 16, True), (4, 20, 20, 32, True)]:
            x = torch.randn(B, Ci, H, W, device=dev).to(dt)
            yw = torch.randn(B, Co, H, m, 2, device=dev) / W
            wc = torch.randn(Co, Ci, device=dev)
            b = torch.randn(Co, device=dev)
            ops.fno_c2r_pw(yw, x, wc, b, gelu)
            t = time_graph(lambda: ops.fno_c2r_pw(yw, x, wc, b, gelu), 20)
            key = f"c2r_pw {tag} B{B} Ci{Ci} Co{Co} m{m} gelu{int(gelu)}"
            res[key] = t
            print(key, f"{t:.1f} us", flush=True)
        for (B, C, m) in [(1, 20, 32), (1, 20, 16), (4, 20, 32)]:
            x = torch.randn(B, C, H, W, device=dev).to(dt)
            ops.dftw_r2c(x, m, 1.0)
            t = time_graph(lambda: ops.dftw_r2c(x, m, 1.0), 20)
            key = f"dftw_r2c {tag} B{B} C{C} m{m}"
            res[key] = t
            print(key, f"{t:.1f} us", flush=True)
    for (B, M) in [(1, 2048), (4, 2048), (32, 2048)]:
        xm = torch.randn(B, 20, M, 2, device=dev)
        w = torch.randn(20, 20, M, 2, device=dev)
        ops.fno_mix(xm, w)
        t = time_graph(lambda: ops.fno_mix(xm, w), 20)
        res[f"fno_mix B{B} M{M}"] = t
        print(f"fno_mix B{B} M{M}", f"{t:.1f} us", flush=True)
    for (B, m) in [(1, 32), (4, 32)]:
        xw = torch.randn(B, 20, H, m, 2, device=dev)
        ops.c2c_axis(xw, 2, H, H, 0, 32, 32, False, 1.0)
        t = time_graph(lambda: ops.c2c_axis(xw, 2, H, H, 0, 32, 32, False, 1.0), 20)
        res[f"c2c_axis fwd B{B}"] = t
        print(f"c2c_axis fwd B{B}", f"{t:.1f} us", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
