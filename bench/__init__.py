"""Benchmarks and kernel studies (not part of the product package)."""


def note_tuning_build(knobs: str) -> None:
    """The A/B switches these sweeps set are read only by a tuning build of the library
    (csrc/ops/tuning.h: MI_DFT_HIPCC_EXTRA=-DAMD_DFT_TUNING=1, loaded via MI_DFT_LIB); say so when
    the loaded library ignores them."""
    import sys

    import torch

    import tensorrt_dft_plugins_amd as tdp

    tdp.load_plugins()
    if not torch.ops.amd_dft.tuning_build():
        print(f"[bench] note: {knobs} are read only by a tuning build (csrc/ops/tuning.h); this library "
              "ignores them, every variant below runs the default kernels", file=sys.stderr, flush=True)
