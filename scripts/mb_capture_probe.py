"""Probe: which fork/join form of the micro-batched AFNO block loop captures into a hipGraph.
usage: python scripts/mb_capture_probe.py {events|waitstream|viacur|nochain}"""
import sys

import torch

sys.path.insert(0, ".")
import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet  # noqa: E402
from tensorrt_dft_plugins_amd.ops import spectral as S  # noqa: E402

mode = sys.argv[1]
tdp.load_plugins()
dev = torch.device("cuda")
m = AFNONet(AFNOConfig(depth=2), backend="amd").to(dev).to(torch.bfloat16).eval()
t = torch.randn(2, 90, 180, 768, device=dev).to(torch.bfloat16)
streams = [torch.cuda.Stream(dev) for _ in range(2)]


def run(t):
    cur = torch.cuda.current_stream()
    ts = list(t.chunk(2))
    pend = [None, None]
    for s in streams:
        s.wait_stream(cur)
    prev_s = None
    prev_e = None
    for blk in m.blocks:
        for i, s in enumerate(streams):
            with torch.cuda.stream(s):
                x, yn = S.afno_block_spectral(blk, ts[i], pend[i])
                if mode == "events" and prev_e is not None:
                    s.wait_event(prev_e)
                if mode == "waitstream" and prev_s is not None and prev_s is not s:
                    s.wait_stream(prev_s)
                if mode == "viacur" and prev_s is not None and prev_s is not s:
                    cur.wait_stream(prev_s)
                    s.wait_stream(cur)
                pend[i] = S.afno_block_mlp(blk, yn)
                if mode == "events":
                    prev_e = torch.cuda.Event()
                    prev_e.record(s)
                prev_s = s
                ts[i] = x
    outs = []
    for i, s in enumerate(streams):
        with torch.cuda.stream(s):
            outs.append(ts[i] + pend[i])
    for s in streams:
        cur.wait_stream(s)
    return torch.cat(outs, 0)


with torch.no_grad():
    s0 = torch.cuda.Stream()
    s0.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s0):
        run(t)
    torch.cuda.current_stream().wait_stream(s0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = run(t)
    g.replay()
    torch.cuda.synchronize()
print(mode, "OK", float(out.float().abs().mean()))
