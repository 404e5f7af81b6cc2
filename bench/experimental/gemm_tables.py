"""[comparator only; moved out of the package in round 3] hipBLASLt solution tables for the FourCastNet MLP GEMMs (PyTorch TunableOp, lookup only).

Measured on MI355X (`scripts/gemm_candidates.py`, `scripts/gemm_forced.py`,
`scripts/interference_probe.py` + `scripts/spin_hog.py`; profiles/gemm_tables_r1o.txt):

* fc2 (in-place ``addmm_``, beta = 1): solution 618613 is 1.77 ms vs 1.86 ms for the default
  heuristic (both data-parallel kernels).
* fc1 (+bias +GELU epilogue): the default is a persistent stream-K kernel (2.59 ms).  Its
  workgroups wait on partial tiles of other workgroups of the same grid, so when another
  long-lived kernel holds even two CUs -- an RCCL collective of the multi-GPU output
  all-gather running on the communication stream -- the whole step slows from 77.5 to 105 ms.
  Solution 618465 (data-parallel, 256x224 tiles) is 2.67 ms and unaffected (80.1 -> 80.1 ms).

So one GPU uses ``fourcastnet_dp1.csv`` (fastest) and data-parallel runs with an overlapped
all-gather use ``fourcastnet_dpN.csv`` (no stream-K).  The tables' validator lines pin the
hipBLASLt / rocBLAS / PyTorch versions and the GPU arch; PyTorch rejects a table that does
not match, and then the default heuristics run.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from tensorrt_dft_plugins_amd.utils.trace import get_logger

TABLE_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuning")
_loaded: Optional[str] = None


def table_for_world(world: int) -> str:
    return os.path.join(TABLE_DIR, "fourcastnet_dp1.csv" if world <= 1 else "fourcastnet_dpN.csv")


def use_gemm_table(path: str) -> bool:
    """Enable TunableOp in lookup-only mode with ``path``; returns True if the table was accepted.
    ``MI_DFT_GEMM_TABLE=0`` disables (hipBLASLt default heuristics)."""
    global _loaded
    if os.environ.get("MI_DFT_GEMM_TABLE", "1") == "0" or not torch.cuda.is_available() or not os.path.isfile(path):
        return False
    if _loaded == path:
        return True
    import torch.cuda.tunable as tunable

    tunable.enable(True)
    tunable.tuning_enable(False)
    tunable.record_untuned_enable(False)
    # results are only read, never written back
    tunable.set_filename(os.path.join("/tmp", f"amd_dft_tunable_unused_{os.getpid()}.csv"))
    ok = bool(tunable.read_file(path))
    log = get_logger("gemm_tables")
    if ok:
        _loaded = path
        log.info("hipBLASLt solution table %s accepted", os.path.basename(path))
    else:
        log.warning("hipBLASLt solution table %s rejected (validator mismatch): default heuristics", path)
    return ok
