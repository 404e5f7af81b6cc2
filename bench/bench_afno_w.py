"""FourCastNet AFNO W-direction transforms (channel-last [32, 90, 180, 768] bf16): the pruned R2C
along W (46 of 91 modes) and the C2R with two fused addends, per fixed-kernel tile config.

Usage: python bench/bench_afno_w.py [--batch 32]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from bench.bench_fft import time_graph  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--cfgs", nargs="+", default=["auto", "15,16", "15,32", "15,64"])
    a = ap.parse_args(argv)
    tdp.load_plugins()
    ops = torch.ops.amd_dft
    B, H, W, C, KM = a.batch, 90, 180, 768, 46
    x = torch.randn(B, H, W, C, device="cuda").to(torch.bfloat16)
    r = torch.randn_like(x)
    s = 1.0 / (H * W) ** 0.5
    yw = ops.r2c(x, [2], s, [KM, 0], torch.bfloat16)
    nbytes_r2c = x.numel() * 2 + yw.numel() * 2
    nbytes_c2r = yw.numel() * 2 + 3 * x.numel() * 2
    res = {}
    for cfg in a.cfgs:
        if cfg == "auto":
            os.environ.pop("MI_DFT_FIXED_CFG", None)
        else:
            os.environ["MI_DFT_FIXED_CFG"] = cfg
        f1 = lambda: ops.r2c(x, [2], s, [KM, 0], torch.bfloat16)  # noqa: E731
        f2 = lambda: ops.c2r_add(yw, [2], [W], s, [KM, 0], x, r, torch.bfloat16)  # noqa: E731
        f1(), f2()
        t1 = min(time_graph(f1, 10) for _ in range(3))
        t2 = min(time_graph(f2, 10) for _ in range(3))
        res[cfg] = {"r2c_us": round(t1, 1), "r2c_TBps": round(nbytes_r2c / t1 / 1e6, 2),
                    "c2r_add_us": round(t2, 1), "c2r_TBps": round(nbytes_c2r / t2 / 1e6, 2)}
        print(cfg, json.dumps(res[cfg]), flush=True)
    os.environ.pop("MI_DFT_FIXED_CFG", None)
    return res


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import note_tuning_build

    note_tuning_build("MI_DFT_FIXED_CFG")
    main()
