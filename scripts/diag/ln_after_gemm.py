"""Is the in-step LN2-split slowdown (850 us in the FourCastNet step vs 530 us standalone) the
state the MLP GEMMs leave the chip in, or a freshly written input?  Times layer_norm_split
eagerly (events around it) right after a bf16x3 fc2 GEMM and/or a 1.6 GB write of its input.
(An earlier run of this script with an idle gap instead: 546-931 us after idle, 522-544 us
right after the GEMM -- the clock ramps, the GEMMs do not throttle the kernel.)"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import tensorrt_dft_plugins_amd as tdp
tdp.load_plugins()
ops = torch.ops.amd_dft
M, C, H = 32 * 16200, 768, 3072
x = torch.randn(M, C, device="cuda")
g, b = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1
hs = ops.split_bf16(torch.randn(M, H, device="cuda") * 0.1)
w2s = ops.split_bf16(torch.randn(C, H, device="cuda") * 0.02)
r = torch.randn(M, C, device="cuda")
ops.layer_norm_split(x, g, b, 1e-6, None); ops.linear3(hs, w2s, None, 0, r, False); torch.cuda.synchronize()


def timed_ln():
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); ops.layer_norm_split(x, g, b, 1e-6, None); e1.record()
    return e0, e1


x2 = torch.randn(M, C, device="cuda")
for mode in ("after_gemm", "after_write", "after_gemm_write", "after_write"):
    ts = []
    for _ in range(5):
        if mode.startswith("after_gemm"):
            for _ in range(3):
                ops.linear3(hs, w2s, None, 0, r, False)
        if mode.endswith("write"):  # the LN input freshly written, as C2R_W + residual does in the step
            x.copy_(x2)
        e0, e1 = timed_ln()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000)
    print(f"{mode:10s} layer_norm_split us: {[round(t) for t in ts]}", flush=True)
