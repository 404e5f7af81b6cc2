"""Large-grid determinism + accuracy screen of every native kernel family (scripts/diag/determinism.py):
workgroups co-resident on the CUs, each op run 3x, bit-identical outputs that match the CPU
(ATen fp32) implementation.  Guards against cross-wave races and co-residency faults such as the gfx950 packed-FP32
op_sel fault beside MFMA waves that once corrupted the AFNO spectral kernels (csrc/spectral/afno_spectral.hip header;
the static guard is tests/test_codegen.py)."""
import os
import runpy

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_kernel_families_deterministic_at_large_grids(device):
    with pytest.raises(SystemExit) as e:
        runpy.run_path(os.path.join(ROOT, "scripts", "diag", "determinism.py"), run_name="__main__")
    assert e.value.code == 0
