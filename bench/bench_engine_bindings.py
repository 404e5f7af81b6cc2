"""execute_v2 latency by binding kind (the reference's TensorRT call, /root/reference/tests/test_dft.py:112-114):
the engine's own buffers, caller-owned device pointers through the copy path, and caller pointers with a graph
bound to them (Engine.BOUND_GRAPH_AFTER / BOUND_GRAPH_MAX).  rfft2 720x1440 fp32 batch 1 engine; per call:
execute_v2 (enqueue + stream synchronize), host wall clock, median of 5 rounds of 200 calls.

  python bench/bench_engine_bindings.py
"""
import os
import statistics
import sys
import time

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from tensorrt_dft_plugins_amd.engine import Engine  # noqa: E402
from tensorrt_dft_plugins_amd.onnx import exporter as ex  # noqa: E402


class Rfft2(nn.Module):
    def forward(self, x):
        return ex.OnnxRfft2.apply(x)


def per_call_us(fn, calls=200, rounds=5):
    for _ in range(20):
        fn()
    res = []
    for _ in range(rounds):
        t0 = time.perf_counter()
        for _ in range(calls):
            fn()
        res.append((time.perf_counter() - t0) / calls * 1e6)
    return statistics.median(res)


def main():
    tdp.load_plugins()
    dev = "cuda"
    eng = Engine.build(Rfft2(), (torch.randn(1, 1, 720, 1440),), device=dev)
    x = torch.randn(1, 1, 720, 1440, device=dev)
    y = torch.empty(1, 1, 720, 721, 2, device=dev)
    eng.binding_tensors[0].copy_(x)
    own = eng.binding_ptrs()
    foreign = [x.data_ptr(), y.data_ptr()]
    r = {"own buffers (main graph)": per_call_us(lambda: eng.execute_v2(own))}
    eng.BOUND_GRAPH_AFTER = 1 << 30  # never bind: every call through the engine buffers
    r["caller pointers, copy path"] = per_call_us(lambda: eng.execute_v2(foreign))
    eng.BOUND_GRAPH_AFTER = 2
    r["caller pointers, bound graph"] = per_call_us(lambda: eng.execute_v2(foreign))
    ref = torch.view_as_real(torch.fft.rfft2(x.double()))
    err = ((y.double() - ref).norm() / ref.norm()).item()
    for k, v in r.items():
        print(f"{k:32s} {v:8.1f} us per execute_v2", flush=True)
    print("bound stats", eng.bound_stats, "rel err", f"{err:.2e}")


if __name__ == "__main__":
    main()
