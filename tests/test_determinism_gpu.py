"""Large-grid determinism + accuracy screen of every native kernel family (scripts/diag/determinism.py):
workgroups co-resident on the CUs, each op run 3x, bit-identical outputs that match the CPU
(ATen fp32) implementation.  Guards against cross-wave races and the co-resident-workgroup corruption that the AMDGPU
load/store vectorizer caused in the AFNO spectral kernels (csrc/spectral/afno_spectral.hip header)."""
import os
import runpy

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_kernel_families_deterministic_at_large_grids(device):
    with pytest.raises(SystemExit) as e:
        runpy.run_path(os.path.join(ROOT, "scripts", "diag", "determinism.py"), run_name="__main__")
    assert e.value.code == 0
