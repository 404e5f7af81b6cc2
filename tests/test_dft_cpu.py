"""CPU-tier tests: registration, op contract, shape inference, validation,
planner factorisation.  The CPU dispatch key runs torch.fft (plumbing; the HIP kernels are
covered by tests/test_dft_gpu.py)."""
import pytest
import torch

import tensorrt_dft_plugins_amd as tdp
from tensorrt_dft_plugins_amd.ops import dft
from helpers import rel_l2


def test_plugins_load():
    # reference: tests/test_dft.py:118-121
    names = tdp.plugin_names()
    assert "Rfft" in names
    assert "Irfft" in names
    c = tdp.get_plugin_creator("Rfft", "1")
    assert [f["name"] for f in c["fields"]] == ["normalized", "onesided", "signal_ndim"]
    assert c["domain"] == "com.microsoft"


def test_load_plugins_idempotent():
    tdp.load_plugins()
    tdp.load_plugins()
    assert tdp.is_loaded()


def test_reference_compat_alias():
    import trt_dft_plugins

    trt_dft_plugins.load_plugins()
    assert "Rfft" in trt_dft_plugins.plugin_names()


@pytest.mark.parametrize("dft_dim1", [1, 2])
@pytest.mark.parametrize("dft_dim2", [4])
@pytest.mark.parametrize("num_c", [1, 3])
@pytest.mark.parametrize("batch_size", [1, 2])
def test_contrib_grid_cpu(dft_dim1, dft_dim2, num_c, batch_size):
    torch.manual_seed(1)
    x = torch.randn(batch_size, num_c, dft_dim1, dft_dim2)
    y = tdp.contrib_rfft(x, signal_ndim=2)
    y_expected = torch.view_as_real(torch.fft.rfft2(x, dim=(-2, -1), norm="backward"))
    assert y.shape == y_expected.shape
    assert torch.allclose(y, y_expected)
    z = tdp.contrib_irfft(y, signal_ndim=2)
    assert torch.allclose(z, torch.fft.irfft2(torch.view_as_complex(y_expected), dim=(-2, -1)))


def test_1d_rfft_1024_cpu_plumbing():
    """BASELINE config 1: 1-D rfft length 1024 batch 1 on CPU."""
    x = torch.randn(1, 1024)
    y = tdp.contrib_rfft(x, signal_ndim=1)
    assert y.shape == (1, 513, 2)
    assert torch.allclose(y, torch.view_as_real(torch.fft.rfft(x)), atol=1e-4)


@pytest.mark.parametrize("signal_ndim", [1, 2, 3])
def test_contrib_shapes(signal_ndim):
    x = torch.randn(2, 3, 6, 8, 10)
    y = tdp.contrib_rfft(x, signal_ndim=signal_ndim)
    assert y.shape == (2, 3, 6, 8, 6, 2)
    z = tdp.contrib_irfft(y, signal_ndim=signal_ndim)
    assert z.shape == x.shape
    assert rel_l2(z, x) < 1e-6


def test_irfft_odd_length_rule():
    # Q9: output length is always 2(m-1)
    x = torch.randn(3, 7)
    y = tdp.contrib_rfft(x, signal_ndim=1)
    assert y.shape[-2] == 4
    assert tdp.contrib_irfft(y, signal_ndim=1).shape[-1] == 6


def test_meta_shapes():
    x = torch.empty(4, 20, 720, 1440, device="meta")
    y = torch.ops.amd_dft.Rfft(x, 0, 1, 2)
    assert y.shape == (4, 20, 720, 721, 2) and y.device.type == "meta"
    z = torch.ops.amd_dft.Irfft(y, 0, 1, 2)
    assert z.shape == (4, 20, 720, 1440)
    p = torch.ops.amd_dft.r2c(x, [2, 3], 1.0, [12, 12, 16, 0])
    assert p.shape == (4, 20, 24, 16, 2)
    q = torch.ops.amd_dft.c2r(p, [2, 3], [720, 1440], 1.0, [12, 12, 16, 0])
    assert q.shape == (4, 20, 720, 1440)


@pytest.mark.parametrize("kw,msg", [({"normalized": 1}, "normalized"), ({"onesided": 0}, "onesided"),
                                    ({"signal_ndim": 0}, "signal_ndim"), ({"signal_ndim": 4}, "signal_ndim")])
def test_attribute_validation(kw, msg):
    x = torch.randn(2, 8, 8, 8, 8)
    args = {"normalized": 0, "onesided": 1, "signal_ndim": 2}
    args.update(kw)
    with pytest.raises(RuntimeError, match=msg):
        torch.ops.amd_dft.Rfft(x, args["normalized"], args["onesided"], args["signal_ndim"])
    with pytest.raises(RuntimeError, match=msg):
        torch.ops.amd_dft.Irfft(torch.randn(2, 8, 8, 5, 2), args["normalized"], args["onesided"], args["signal_ndim"])


def test_rank_limit():
    with pytest.raises(RuntimeError, match="rank"):
        tdp.contrib_rfft(torch.randn(*([2] * 8)), signal_ndim=1)


def test_unsupported_dtype():
    with pytest.raises(RuntimeError, match="unsupported dtype"):
        tdp.contrib_rfft(torch.randn(4, 8, dtype=torch.float64), signal_ndim=1)


def test_torch_fft_api_cpu():
    x = torch.randn(3, 10, 12)
    assert rel_l2(tdp.rfft2(x), torch.fft.rfft2(x.double())) < 1e-6
    assert rel_l2(tdp.rfftn(x, dim=(0, 2), norm="ortho"), torch.fft.rfftn(x.double(), dim=(0, 2), norm="ortho")) < 1e-6
    y = torch.fft.rfft(x)
    assert rel_l2(tdp.irfft(y, n=12), torch.fft.irfft(y.to(torch.complex128), n=12)) < 1e-6
    c = torch.randn(4, 9, dtype=torch.complex64)
    assert rel_l2(tdp.fft(c), torch.fft.fft(c.to(torch.complex128))) < 1e-6
    assert rel_l2(tdp.ifft(c, norm="ortho"), torch.fft.ifft(c.to(torch.complex128), norm="ortho")) < 1e-6
    assert rel_l2(tdp.fft(x[0], n=16), torch.fft.fft(x[0].double(), n=16)) < 1e-6


def test_bf16_cpu():
    x = torch.randn(2, 16, 16).to(torch.bfloat16)
    y = tdp.rfft2(x)
    assert rel_l2(y, torch.fft.rfft2(x.double())) < 1e-6


def test_pruned_cpu():
    torch.manual_seed(0)
    x = torch.randn(2, 3, 32, 40)
    y = dft.rfftn_pruned(x, [2, 3], [(5, 4), (7, 0)])
    full = torch.fft.rfft2(x.double())
    ref = torch.cat([full[:, :, :5, :7], full[:, :, -4:, :7]], dim=2)
    assert rel_l2(torch.view_as_complex(y.contiguous()), ref) < 1e-6
    z = dft.irfftn_pruned(y, [2, 3], [32, 40], [(5, 4), (7, 0)])
    pad = torch.zeros(2, 3, 32, 21, dtype=torch.complex128)
    pad[:, :, :5, :7] = ref[:, :, :5]
    pad[:, :, -4:, :7] = ref[:, :, 5:]
    assert rel_l2(z, torch.fft.irfft2(pad, s=(32, 40))) < 1e-6


def test_planner_factorisation():
    import re

    for n in list(range(1, 300)) + [720, 1440, 1024, 4096, 103, 721, 5000]:
        info = torch.ops.amd_dft.plan_info(n)
        rad = [int(v) for v in re.search(r"radices=\[([0-9,]*)\]", info).group(1).split(",") if v]
        prod = 1
        for r in rad:
            prod *= r
        assert prod == n, (n, info)
        assert len(rad) <= 16
    # FourCastNet sizes use the radix orders of their fixed kernels: 720 = 8x9x10 (three passes), 1440 rows =
    # 5x6x6x8 (four passes of one 5..8-point butterfly per thread at 288 threads, profiles/fft_plans_r3.txt)
    assert "radices=[8,9,10]" in torch.ops.amd_dft.plan_info(720)
    assert "radices=[5,6,6,8]" in torch.ops.amd_dft.plan_info(1440)


def test_utils_runtime_helpers():
    from tensorrt_dft_plugins_amd.utils import check_finite, env_report

    assert "torch" in env_report()
    check_finite(torch.ones(3))
    with pytest.raises(FloatingPointError):
        check_finite(torch.tensor([1.0, float("nan")]))
