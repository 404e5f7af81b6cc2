"""Graph capture with a live RCCL (backend "nccl") process group: the multi-GPU bench captures
its per-step hipGraph after init_process_group, while the NCCL watchdog thread polls events.
A one-GPU box cannot run RCCL across GPUs, but a world-size-1 RCCL communicator exercises the
same capture-vs-watchdog interaction plus all_gather_into_tensor on a side stream.

  python scripts/rccl_capture_probe.py      (MASTER_ADDR/PORT default to 127.0.0.1:29533)
"""
import os
import sys

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    import tensorrt_dft_plugins_amd as tdp
    from tensorrt_dft_plugins_amd.engine.capture import CapturedModule
    from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet

    tdp.load_plugins()
    cfg = AFNOConfig(depth=2)
    model = AFNONet(cfg, backend="amd").cuda().to(torch.bfloat16).eval()
    x = torch.randn(4, cfg.in_chans, *cfg.img_size, device="cuda").to(torch.bfloat16)
    cap = CapturedModule(model, [x], warmup=2, n_graphs=2, use_graph=True)
    comm = torch.cuda.Stream()
    outs = [torch.empty_like(cap.outputs[i][0]) for i in range(2)]
    works = [None, None]
    for k in range(6):
        i = k % 2
        if works[i] is not None:
            works[i].wait()
        o = cap.replay(i)[0]
        ev = torch.cuda.Event()
        ev.record()
        with torch.cuda.stream(comm):
            comm.wait_event(ev)
            works[i] = dist.all_gather_into_tensor(outs[i], o, async_op=True)
    for w in works:
        w.wait()
    torch.cuda.synchronize()
    with torch.no_grad():
        ref = model(x)
    err = ((outs[1].float() - ref.float()).norm() / ref.float().norm()).item()
    print(f"rccl capture probe ok: replay+gather vs eager rel {err:.2e}")
    assert err < 1e-2
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
