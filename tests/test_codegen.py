"""Code-generation guard for the AFNO spectral kernels (CPU tier: hipcc cross-compiles gfx950 here).

The -O3 load/store vectorizer made both AFNO kernels nondeterministically wrong at co-resident grids; the round-3
bisection (profiles/afno_o3_bisect_r3.txt) pinned the trigger to the pass-1 twiddle multiply issued as
`v_pk_mul_f32 vD, vA, vB op_sel:[0,1]` on an LDS-loaded twiddle pair.  This test compiles afno_spectral.hip with the
shipped per-file flags and with the vectorizer on and checks the device code contains no such instruction
(scripts/diag/opsel_lds_check.py); and disassembles every kernel of the built library (scripts/diag/scan_so.py):
none may issue a packed-FP32 op with src1's high half via op_sel -- on MI355X those return wrong products while
another wave on the same SIMD runs MFMAs (scripts/diag/opsel_lds_repro.hip)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts", "diag"))
HIPCC = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")


def _compile(tmp_path, extra):
    from tensorrt_dft_plugins_amd import _build

    src = os.path.join(ROOT, "csrc", "spectral", "afno_spectral.hip")
    out = tmp_path / "afno.s"
    cmd = [HIPCC, "-S", "--cuda-device-only", "-std=c++17", "-O3", "-x", "hip", f"--offload-arch={_build.ARCH}",
           "-munsafe-fp-atomics", "-fno-slp-vectorize", "-I", os.path.join(ROOT, "csrc")]
    cmd += _build._file_flags(src) + extra + [src, "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    return str(out)


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None, reason="hipcc not available")
def test_afno_kernels_emit_no_src1_high_packed_fp32(tmp_path):
    """afno_spectral.hip with its shipped flags AND with the vectorizer on (the build that used to go wrong) emits no
    packed-FP32 op taking src1's high half via op_sel (radix.h c_mul routes the twiddle's imaginary part through
    its own register); the scanner itself is checked on the minimal reproducer, which issues the form on purpose."""
    import opsel_lds_check as chk

    for extra in ([], ["-mllvm", "-amdgpu-load-store-vectorizer=1"]):
        r = chk.scan(_compile(tmp_path, extra))
        assert r and sum(t for _, t in r.values()) == 0, (extra, {k: v for k, v in r.items() if v[1]})
    out = tmp_path / "repro.s"
    subprocess.run([HIPCC, "-S", "--cuda-device-only", "-O3", "--offload-arch=gfx950",
                    os.path.join(ROOT, "scripts", "diag", "opsel_lds_repro.hip"), "-o", str(out)],
                   check=True, capture_output=True, timeout=600)
    assert sum(l for l, _ in chk.scan(str(out)).values()) > 0, "scanner no longer sees the form in the reproducer"


# the library under test: MI_DFT_LIB when set (CI builds elsewhere and points both tiers at it), else the in-tree
# one -- the same rule tensorrt_dft_plugins_amd/_loader.py uses, so the scan inspects the binary the tests load
SO = os.environ.get("MI_DFT_LIB") or os.path.join(ROOT, "tensorrt_dft_plugins_amd", "_C.so")


@pytest.mark.skipif(not os.path.exists(SO), reason="library not built")
def test_no_kernel_mixes_mfma_with_src1_high_packed_fp32():
    """Every gfx950 kernel in the shipped library: none contains both an MFMA and a packed-FP32 instruction that
    takes the high half of src1 via op_sel -- on MI355X the latter returns wrong results while another wave on the
    same SIMD runs MFMAs (scripts/diag/opsel_lds_repro.hip: 7.7 % of products; src0 op_sel and no op_sel are
    unaffected).  The kernels that do contain the packed form (AFNO W-transforms) contain no MFMA."""
    import scan_so

    r = scan_so.scan(SO)
    assert len(r) > 100 and sum(1 for v in r.values() if v[0]) > 10, "disassembly found too few kernels"
    both = {k: v for k, v in r.items() if v[0] and v[1]}
    assert not both, both
    # stronger, since radix.h's c_mul stopped producing it: no kernel issues the form at all (a kernel without MFMA
    # could still share a SIMD with another stream's MFMA kernel)
    with_form = {k: v for k, v in r.items() if v[1]}
    assert not with_form, with_form
