"""The opt-in hand-GEMM epilogue variant against the default kernel, each in its own process (the
variant is read once per process): MI_DFT_GEMM_EPI=direct (epilogue stored straight from the MFMA
layout).  (The 4-wave / two-workgroup kernels moved to bench/experimental/ in round 3; the
start-stagger experiment was removed in round 4.)

Same MFMA order per accumulator in every variant, so bf16 outputs must match exactly and the
fp32 / split-pair outputs to fp32 rounding (the epilogues contract their FMAs differently).
Launches: fc1 + GELU (split-pair out) -> fc2 + fp32 residual, plain fc1 (fp32 out), and the
bf16 fc1 + GELU -> fc2 + bf16 residual, at a ragged M (bench/gemm_variant_ab.py CHILD)."""
import os
import subprocess
import sys

import pytest
import torch

from helpers import rel_l2

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, name, env_extra):
    from bench.gemm_variant_ab import CHILD

    f = str(tmp_path / f"{name}.pt")
    env = dict(os.environ, **env_extra)
    subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT}, f], env=env, check=True, timeout=240)
    return torch.load(f, weights_only=True)


@pytest.mark.gpu
def test_gemm_persistent_matches_default(device, tmp_path):
    """MI_DFT_GEMM_PERSIST=1: the FourCastNet block GEMMs on a persistent grid (next tile's first
    K-tile streamed in under the epilogue, counted waits across it) -- same MFMA order and epilogue
    arithmetic, so every output must be bit-identical, the ragged last token tile included; the LN
    partial statistics ('part') are summed in another order there (16-lane DPP sums instead of the
    default's per-row sweeps) and agree to fp32 rounding."""
    base = _run(tmp_path, "default", {"MI_DFT_GEMM_PERSIST": "0"})
    other = _run(tmp_path, "persist", {"MI_DFT_GEMM_PERSIST": "1"})
    for k in base:
        if k == "part":
            assert torch.allclose(base[k], other[k], rtol=1e-5, atol=1e-5), (base[k] - other[k]).abs().max()
        else:
            assert torch.equal(base[k], other[k]), (k, (base[k].float() - other[k].float()).abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [{"MI_DFT_GEMM_EPI": "direct"}], ids=["direct-epilogue"])
def test_gemm_variant_matches_default(device, tmp_path, variant):
    from tensorrt_dft_plugins_amd.ops.spectral import unsplit_bf16

    base = _run(tmp_path, "default", {"MI_DFT_GEMM_EPI": "staged"})
    other = _run(tmp_path, "variant", variant)
    for k in ("hb", "yb"):  # bf16 outputs: identical arithmetic
        assert torch.equal(base[k], other[k]), k
    assert rel_l2(unsplit_bf16(other["h"]), unsplit_bf16(base["h"])) < 1e-6
    for k in ("y", "y1"):
        assert rel_l2(other[k], base[k]) < 1e-6, k
    # (the fp32 block's GEMMs always use the staged epilogue: hl / ys / part / yp are not compared)
