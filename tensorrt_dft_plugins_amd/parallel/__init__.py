"""Parallelism: batch data-parallel inference over RCCL (xGMI) / Gloo."""
from .dp import DataParallelInference, all_gather_batch, init_distributed, world_info  # noqa: F401
from .streams import MicroBatchStreams  # noqa: F401,E402
