"""Parallelism: batch data-parallel inference over RCCL (xGMI) / Gloo, slab-decomposed 2-D FFT."""
from .dp import DataParallelInference, all_gather_batch, init_distributed, world_info  # noqa: F401
from .ipc_gather import IpcAllGather, ShmTransport  # noqa: F401,E402
from .slab_fft import h_slab, k_slab, slab_irfft2, slab_rfft2  # noqa: F401,E402
