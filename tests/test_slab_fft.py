"""Slab-decomposed distributed rfft2 / irfft2 (parallel/slab_fft.py): rows local -> all_to_all
transpose -> columns local.  CPU tier: world 1 in-process, Gloo world 2 and 3 (uneven slabs)
against torch.fft on the full field."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _field(shape, seed=0):
    return torch.randn(*shape, generator=torch.Generator().manual_seed(seed))


@pytest.mark.parametrize("norm", [None, "ortho", "forward"])
def test_slab_fft_single_rank(norm):
    from tensorrt_dft_plugins_amd.parallel import slab_irfft2, slab_rfft2

    x = _field((2, 3, 10, 16))
    y = slab_rfft2(x, 10, norm=norm)
    ref = torch.fft.rfft2(x, norm=norm)
    torch.testing.assert_close(y, ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(slab_irfft2(y, 16, norm=norm), x, rtol=1e-4, atol=1e-4)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, H, W, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        sys.path.insert(0, ROOT)
        import torch.distributed as dist

        from tensorrt_dft_plugins_amd.parallel import h_slab, k_slab, slab_irfft2, slab_rfft2

        dist.init_process_group("gloo", rank=rank, world_size=world)
        x = _field((2, H, W), seed=7)  # same full field everywhere; each rank keeps its slab
        h0, h1 = h_slab(H, world, rank)
        y = slab_rfft2(x[:, h0:h1].contiguous(), H, norm="ortho")
        k0, k1 = k_slab(W // 2 + 1, world, rank)
        ref = torch.fft.rfft2(x, norm="ortho")[:, :, k0:k1]
        err_f = ((y - ref).abs().max() / ref.abs().max()).item()
        xb = slab_irfft2(y, W, norm="ortho")
        err_b = ((xb - x[:, h0:h1]).abs().max()).item()
        q.put((rank, err_f, err_b, tuple(y.shape), tuple(xb.shape)))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:
        q.put((rank, repr(e), None, None, None))
        raise


@pytest.mark.parametrize("world,H,W", [(2, 12, 20), (3, 10, 18)])
def test_slab_fft_gloo(world, H, W):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, H, W, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    from tensorrt_dft_plugins_amd.parallel import h_slab, k_slab

    for rank, err_f, err_b, ys, xs in res:
        assert not isinstance(err_f, str), err_f
        assert err_f < 1e-5 and err_b < 1e-4, (rank, err_f, err_b)
        k0, k1 = k_slab(W // 2 + 1, world, rank)
        h0, h1 = h_slab(H, world, rank)
        assert ys == (2, H, k1 - k0) and xs == (2, h1 - h0, W)


@pytest.mark.gpu
def test_slab_fft_single_rank_gpu(device):
    """The slab path's local passes on the HIP kernels (720 x 1440, one rank)."""
    from tensorrt_dft_plugins_amd.parallel import slab_irfft2, slab_rfft2

    x = _field((1, 720, 1440), seed=3)
    y = slab_rfft2(x.to(device), 720, norm="ortho")
    ref = torch.fft.rfft2(x.double(), norm="ortho")
    assert ((y.cpu().to(torch.complex128) - ref).abs().max() / ref.abs().max()).item() < 1e-5
    xb = slab_irfft2(y, 1440, norm="ortho").cpu()
    assert (xb - x).abs().max().item() < 1e-4
