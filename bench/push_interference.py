"""IPC direct-push interference on one GPU: step time of the captured
FourCastNet forward alone vs. with the ``ipc_push`` kernel (csrc/parallel/ipc_push.hip) copying
the previous step's output on a second stream at the same time -- the overlap the IPC gather
runs in multi-GPU DP.  The peers are stood in for by local buffers, so the push's writes land in
this GPU's HBM instead of going out over xGMI (an upper bound on the interference: in DP only
the shard reads stay local).

Usage: python bench/push_interference.py [--dtype fp32|bf16] [--batch 32] [--ndst 1,3] [--steps 6]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from tensorrt_dft_plugins_amd.engine.capture import CapturedModule  # noqa: E402
from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--ndst", default="1,3")
    ap.add_argument("--steps", type=int, default=6)
    a = ap.parse_args()
    tdp.load_plugins()
    dt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    torch.manual_seed(1234)
    cfg = AFNOConfig()
    m = AFNONet(cfg, backend="amd").cuda().to(dt).eval()
    x = torch.randn(a.batch, cfg.in_chans, *cfg.img_size, device="cuda").to(dt)
    cap = CapturedModule(m, [x], warmup=2, n_graphs=2)
    side = torch.cuda.Stream()
    ops = torch.ops.amd_dft

    def run(ndst):
        dsts = [torch.empty_like(cap.outputs[0][0]) for _ in range(ndst)]
        ptrs = [d.data_ptr() for d in dsts]
        for _ in range(2):
            cap.replay(0)
        torch.cuda.synchronize()
        ts = []
        for k in range(a.steps):
            ev = torch.cuda.Event()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out_prev = cap.outputs[(k + 1) % 2][0]
            if ndst:
                ev.record()
                with torch.cuda.stream(side):
                    side.wait_event(ev)
                    ops._ipc_push(out_prev, ptrs, 0)  # previous step's output, while this step computes
            cap.replay(k % 2)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        return ts[len(ts) // 2], dsts

    base, _ = run(0)
    shard_gb = cap.outputs[0][0].numel() * cap.outputs[0][0].element_size() / 1e9
    print(f"{a.dtype} batch {a.batch}: step alone {base:.2f} ms (output shard {shard_gb:.2f} GB)", flush=True)
    for n in [int(v) for v in a.ndst.split(",")]:
        t, dsts = run(n)
        ok = all(torch.equal(d, cap.outputs[0][0]) or torch.equal(d, cap.outputs[1][0]) for d in dsts)
        print(f"  + concurrent ipc_push of the previous output to {n} local buffer(s): {t:.2f} ms "
              f"({(t / base - 1) * 100:+.1f} %), copies intact: {ok}", flush=True)
    again, _ = run(0)
    print(f"step alone again {again:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
