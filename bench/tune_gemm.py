"""PyTorch TunableOp search over the hipBLASLt/rocBLAS solutions for the FourCastNet MLP GEMMs
(fc1 768->3072 + bias + GELU, fc2 3072->768 + bias, M = batch*16200 tokens, bf16).

    python bench/tune_gemm.py --out tensorrt_dft_plugins_amd/tuned/gemm_mi355x.csv

Prints the default-heuristic time, tunes (TunableOp benchmarks every candidate solution per
GEMM shape), then prints the tuned time; the winning solutions land in the CSV that
`tensorrt_dft_plugins_amd.utils.gemm_tuning` loads at run time."""
import argparse
import os
import statistics
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--out", default="gpurun_out/tunableop_results.csv")
    ap.add_argument("--max-ms", type=int, default=400, help="tuning time budget per GEMM shape")
    a = ap.parse_args()
    M, C, Hd = a.batch * 16200, 768, 3072
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(M, C, device=dev, dtype=torch.bfloat16, generator=g)
    w1 = torch.randn(Hd, C, device=dev, dtype=torch.bfloat16, generator=g) * 0.02
    b1 = torch.randn(Hd, device=dev, dtype=torch.bfloat16, generator=g) * 0.02
    w2 = torch.randn(C, Hd, device=dev, dtype=torch.bfloat16, generator=g) * 0.02
    b2 = torch.randn(C, device=dev, dtype=torch.bfloat16, generator=g) * 0.02
    h = F.gelu(F.linear(x, w1, b1))
    cases = {
        "fc1 addmm_act gelu": lambda: torch._addmm_activation(b1, x, w1.t(), use_gelu=True),
        "fc1 linear": lambda: F.linear(x, w1, b1),
        "fc2 linear": lambda: F.linear(h, w2, b2),
    }
    flops = {"fc1 addmm_act gelu": 2 * M * C * Hd, "fc1 linear": 2 * M * C * Hd, "fc2 linear": 2 * M * C * Hd}
    base = {k: timed(f) for k, f in cases.items()}
    for k, v in base.items():
        print(f"default  {k:20s} {v:8.3f} ms  {flops[k] / v / 1e9:7.1f} TFLOP/s", flush=True)

    tun = torch.cuda.tunable
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    tun.set_filename(a.out)
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(a.max_ms)
    tun.set_max_tuning_iterations(30)
    t0 = time.time()
    for k, f in cases.items():
        f()
        torch.cuda.synchronize()
        print(f"tuned {k} ({time.time() - t0:.1f} s)", flush=True)
    tun.tuning_enable(False)
    tun.write_file()
    for k, f in cases.items():
        v = timed(f)
        print(f"tuned    {k:20s} {v:8.3f} ms  {flops[k] / v / 1e9:7.1f} TFLOP/s  ({base[k] / v:.3f}x)", flush=True)
    print("results:", tun.get_results())


if __name__ == "__main__":
    main()
