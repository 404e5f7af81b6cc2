"""ONNX tier: export (contrib Rfft/Irfft nodes), protobuf schema, importer/executor.

Port of the reference pipeline (/root/reference/tests/test_dft.py:124-184: torch -> ONNX ->
TensorRT plan -> run -> allclose) with the TensorRT parser/builder replaced by this library's
ONNX importer; runs on CPU here and on the MI355X in the GPU tier.
"""
import io

import pytest
import torch
import torch.nn as nn

import tensorrt_dft_plugins_amd as tdp
from tensorrt_dft_plugins_amd.onnx import exporter as ex
from tensorrt_dft_plugins_amd.onnx import proto as P
from tensorrt_dft_plugins_amd.onnx.runner import OnnxGraph, supported_ops


class RfftModel(nn.Module):
    def forward(self, x):
        return ex.OnnxRfft2.apply(x)


class IrfftModel(nn.Module):
    def forward(self, x):
        return ex.OnnxIrfft2.apply(x)


def _node_summary(data: bytes):
    m = P.load_model(data)
    return m, [(n.op_type, n.domain, {a.name: a.i for a in n.attribute}) for n in m.graph.node]


def test_export_contrib_node_bytes():
    data = ex.export(RfftModel(), torch.randn(2, 3, 2, 4))
    m, nodes = _node_summary(data)
    assert nodes == [("Rfft", "com.microsoft", {"normalized": 0, "onesided": 1, "signal_ndim": 2})]
    opsets = {o.domain: o.version for o in m.opset_import}
    assert opsets[""] == 15 and opsets["com.microsoft"] == 1
    # attributes are INT typed (TensorRT PluginField kINT32 parity)
    assert all(a.type == P.ATTR_INT for a in m.graph.node[0].attribute)


def test_export_direct_custom_op_call():
    class M(nn.Module):
        def forward(self, x):
            return tdp.contrib_irfft(tdp.contrib_rfft(x, signal_ndim=1) * 2.0, signal_ndim=1)

    data = ex.export(M(), torch.randn(3, 16))
    _, nodes = _node_summary(data)
    kinds = [(n[0], n[1]) for n in nodes]
    assert ("Rfft", "com.microsoft") in kinds and ("Irfft", "com.microsoft") in kinds


@pytest.mark.parametrize("dft_dim1", [1, 2])
@pytest.mark.parametrize("dft_dim2", [4])
@pytest.mark.parametrize("num_c", [1, 3])
@pytest.mark.parametrize("batch_size", [1, 2])
def test_rfft2_pipeline_cpu(dft_dim1, dft_dim2, num_c, batch_size):
    torch.manual_seed(1)
    x = torch.randn(batch_size, num_c, dft_dim1, dft_dim2)
    onnx_model = ex.export(RfftModel(), x)
    g = OnnxGraph(onnx_model, device="cpu")
    y_expected = torch.view_as_real(torch.fft.rfft2(x, dim=(-2, -1), norm="backward"))
    (y,) = g.run(x)
    assert torch.allclose(y_expected, y)


@pytest.mark.parametrize("dft_dim1", [1, 2])
@pytest.mark.parametrize("dft_dim2", [4])
@pytest.mark.parametrize("num_c", [1, 3])
@pytest.mark.parametrize("batch_size", [1, 2])
def test_irfft2_pipeline_cpu(dft_dim1, dft_dim2, num_c, batch_size):
    torch.manual_seed(1)
    x = torch.randn(batch_size, num_c, dft_dim1, dft_dim2)
    y = torch.view_as_real(torch.fft.rfft2(x))
    onnx_model = ex.export(IrfftModel(), y)
    g = OnnxGraph(onnx_model, device="cpu")
    x_expected = torch.fft.irfft2(torch.view_as_complex(y), dim=(-2, -1))
    (x_actual,) = g.run(y)
    assert torch.allclose(x_expected, x_actual, atol=1e-6)


@pytest.mark.parametrize("nd", [1, 2, 3])
def test_signal_ndim_roundtrip(nd):
    class M(nn.Module):
        def forward(self, x):
            return ex.irfft(ex.rfft(x, nd) * 0.5, nd)

    x = torch.randn(2, 4, 6, 8)
    g = OnnxGraph(ex.export(M(), x), device="cpu")
    (z,) = g.run(x)
    assert torch.allclose(z, 0.5 * x, atol=1e-5)


def test_invalid_attributes_rejected_at_build():
    m = P.ModelProto()
    m.ir_version = 8
    op = m.opset_import.add()
    op.domain, op.version = "com.microsoft", 1
    gi = m.graph.input.add()
    gi.name = "x"
    gi.type.tensor_type.elem_type = P.FLOAT
    n = m.graph.node.add()
    n.op_type, n.domain = "Rfft", "com.microsoft"
    n.input.append("x")
    n.output.append("y")
    for k, v in (("normalized", 1), ("onesided", 1), ("signal_ndim", 2)):
        a = n.attribute.add()
        a.name, a.i, a.type = k, v, P.ATTR_INT
    m.graph.output.add().name = "y"
    with pytest.raises(ValueError, match="invalid Rfft attributes"):
        OnnxGraph(m.SerializeToString(), device="cpu")


def test_unknown_op_message():
    m = P.ModelProto()
    n = m.graph.node.add()
    n.op_type = "NoSuchOp"
    with pytest.raises(NotImplementedError, match="NoSuchOp"):
        OnnxGraph(m, device="cpu")


def test_standard_onnx_dft_op():
    from tensorrt_dft_plugins_amd.onnx.runner import _OPS

    x = torch.randn(2, 12, 1)
    y = _OPS[("", "DFT")]({"onesided": 1, "axis": 1}, x)
    assert torch.allclose(torch.view_as_complex(y.contiguous()), torch.fft.rfft(x[..., 0], dim=1), atol=1e-5)
    c = torch.randn(2, 10, 2)
    z = _OPS[("", "DFT")]({"inverse": 1, "axis": 1}, c)
    assert torch.allclose(torch.view_as_complex(z.contiguous()), torch.fft.ifft(torch.view_as_complex(c), dim=1),
                          atol=1e-5)


def test_generic_model_ops_roundtrip():
    """An FNO-flavoured graph with standard ops (Conv, GELU, LayerNorm, Einsum, Slice, ...)."""

    class M(nn.Module):
        def __init__(self):
            super().__init__()
            self.conv = nn.Conv2d(3, 8, 1)
            self.ln = nn.LayerNorm(16)
            self.w = nn.Parameter(torch.randn(8, 8, 4, 9, 2) * 0.1)

        def forward(self, x):
            h = self.ln(torch.nn.functional.gelu(self.conv(x)))
            f = ex.rfft(h, 2)
            f = f[:, :, :4, :9]
            fr, fi = f[..., 0], f[..., 1]
            wr, wi = self.w[..., 0], self.w[..., 1]
            o = torch.stack([torch.einsum("bixy,ioxy->boxy", fr, wr) - torch.einsum("bixy,ioxy->boxy", fi, wi),
                             torch.einsum("bixy,ioxy->boxy", fr, wi) + torch.einsum("bixy,ioxy->boxy", fi, wr)], -1)
            full = torch.zeros(o.shape[0], 8, 16, 9, 2)
            full = torch.cat([o, torch.zeros(o.shape[0], 8, 12, 9, 2)], dim=2)
            return ex.irfft(full, 2) + h

    torch.manual_seed(0)
    m = M().eval()
    x = torch.randn(2, 3, 16, 16)
    with torch.no_grad():
        ref = m(x)
    g = OnnxGraph(ex.export(m, x), device="cpu")
    (y,) = g.run(x)
    assert torch.allclose(y, ref, atol=1e-4)


def test_supported_ops_listing():
    ops = supported_ops()
    assert "com.microsoft::Rfft" in ops and "com.microsoft::Irfft" in ops and "DFT" in ops


def test_export_fast_fno_model_amd_nodes():
    """The MI355X FNO path (native spectral ops) exports as com.amd.dft nodes and re-imports."""
    from tensorrt_dft_plugins_amd.models import FNO2d, FNOConfig
    from tensorrt_dft_plugins_amd.onnx import proto as P

    torch.manual_seed(0)
    cfg = FNOConfig(img_size=(16, 24), in_chans=3, out_chans=2, width=8, modes1=3, modes2=4, n_layers=2,
                    proj_hidden=16)
    m = FNO2d(cfg, backend="amd").eval()
    x = torch.randn(2, 3, 16, 24)
    with torch.no_grad():
        ref = m(x)
    data = ex.export(m, x)
    model = P.load_model(data)
    doms = {n.domain for n in model.graph.node}
    assert "com.amd.dft" in doms
    ops = {n.op_type for n in model.graph.node if n.domain == "com.amd.dft"}
    assert {"dftw_r2c", "c2c_axis", "fno_mix_c2c", "fno_c2r_pw", "fno_pointwise"} <= ops
    (y,) = OnnxGraph(data, device="cpu").run(x)
    assert torch.allclose(y, ref, atol=1e-5)


def test_export_fast_afno_model_amd_nodes():
    from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet

    torch.manual_seed(1)
    cfg = AFNOConfig(img_size=(32, 64), in_chans=3, out_chans=3, embed_dim=64, depth=2, num_blocks=4, patch_size=8)
    m = AFNONet(cfg, backend="amd").eval()
    x = torch.randn(1, 3, 32, 64)
    with torch.no_grad():
        ref = m(x)
    data = ex.export(m, x)
    (y,) = OnnxGraph(data, device="cpu").run(x)
    assert torch.allclose(y, ref, atol=1e-4)


def test_constant_subgraphs_folded_at_load():
    """Nodes whose inputs are all constants run once when the graph is loaded (TensorRT-style
    constant folding): the weight-only subgraph disappears from the per-run node list."""

    class M(nn.Module):
        def __init__(self):
            super().__init__()
            self.w = nn.Parameter(torch.randn(8, 8))

        def forward(self, x):
            w2 = torch.tanh(self.w * 2.0).t()  # constant-only: folded
            return x @ w2 + 1.0

    torch.manual_seed(0)
    m = M().eval()
    x = torch.randn(4, 8)
    with torch.no_grad():
        ref = m(x)
    data = ex.export(m, x)
    g = OnnxGraph(data, device="cpu")
    assert g.folded >= 2
    assert all(op not in ("Tanh", "Transpose", "Mul") for *_, op in g.nodes)
    (y,) = g.run(x)
    assert torch.allclose(y, ref, atol=1e-6)


def test_slice_negative_step_end_minus_one():
    """ONNX Slice with a negative step: end = -1 means index n - 1 after the n is added,
    so starts=[-1], ends=[-1], steps=[-1] is empty; a very negative end walks down past index 0."""
    from tensorrt_dft_plugins_amd.onnx.runner import _slice

    x = torch.arange(6.0)
    t = lambda v: torch.tensor(v, dtype=torch.int64)  # noqa: E731
    assert _slice({}, x, t([-1]), t([-1]), t([0]), t([-1])).numel() == 0
    assert _slice({}, x, t([-1]), t([-(2 ** 63) + 1]), t([0]), t([-1])).tolist() == [5, 4, 3, 2, 1, 0]
    assert _slice({}, x, t([4]), t([1]), t([0]), t([-2])).tolist() == [4, 2]
    assert _slice({}, x, t([-2]), t([-5]), t([0]), t([-1])).tolist() == [4, 3, 2]


def test_large_host_constant_device_copy_released_with_it():
    """The device copy of a large host constant lives exactly as long as the host tensor (its
    graph's constant), not for the process."""
    import gc

    from tensorrt_dft_plugins_amd.onnx import runner as R

    t = torch.arange(10000)
    d = R._to_dev(t, torch.device("meta"))  # any other device: a distinct copy object
    assert d is not t and R._to_dev(t, torch.device("meta")) is d  # memoised while alive
    n = len(R._DEV_LARGE)
    del t, d
    gc.collect()
    assert len(R._DEV_LARGE) == n - 1
