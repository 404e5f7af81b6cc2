"""Engine tier: build / serialise / deserialise / execute (TensorRT plan analogue), CLI parity."""
import os

import pytest
import torch
import torch.nn as nn

from tensorrt_dft_plugins_amd.engine import ENGINE_MAGIC, Engine
from tensorrt_dft_plugins_amd.engine import cli
from tensorrt_dft_plugins_amd.onnx import exporter as ex


class Rfft2Model(nn.Module):
    def forward(self, x):
        return ex.OnnxRfft2.apply(x)


class RoundTrip(nn.Module):
    def forward(self, x):
        return ex.OnnxIrfft2.apply(ex.OnnxRfft2.apply(x) * 0.25)


def _dev(request):
    return request.param


def test_engine_build_run_cpu():
    x = torch.randn(2, 3, 8, 12)
    eng = Engine.build(Rfft2Model(), (x,), device="cpu")
    (y,) = eng.infer(x)
    assert torch.allclose(y, torch.view_as_real(torch.fft.rfft2(x)), atol=1e-5)
    assert [b.name for b in eng.bindings if b.is_input] == eng.input_names
    assert eng.bindings[-1].shape == [2, 3, 8, 7, 2]


def test_engine_serialize_roundtrip_cpu(tmp_path):
    x = torch.randn(1, 2, 16, 16)
    eng = Engine.build(RoundTrip(), (x,), device="cpu")
    p = tmp_path / "rt.engine"
    eng.save(str(p))
    data = open(p, "rb").read()
    assert data.startswith(ENGINE_MAGIC)
    eng2 = Engine.load(str(p), device="cpu")
    (z,) = eng2.infer(x)
    assert torch.allclose(z, 0.25 * x, atol=1e-5)
    assert eng2.header.plugin_version == "1"


def test_engine_execute_v2_host_pointers_cpu():
    x = torch.randn(1, 1, 4, 8)
    eng = Engine.build(Rfft2Model(), (x,), device="cpu")
    y = torch.empty(1, 1, 4, 5, 2)
    assert eng.execute_v2([x.data_ptr(), y.data_ptr()])
    assert torch.allclose(y, torch.view_as_real(torch.fft.rfft2(x)), atol=1e-5)


def test_engine_rejects_bad_file():
    with pytest.raises(ValueError, match="magic"):
        Engine.deserialize(b"not an engine")


def test_engine_static_shape_enforced():
    x = torch.randn(1, 1, 4, 8)
    eng = Engine.build(Rfft2Model(), (x,), device="cpu")
    with pytest.raises(ValueError, match="static"):
        eng.infer(torch.randn(2, 1, 4, 8))


def test_dftexec_cli_build_and_load(tmp_path, capsys):
    x = torch.randn(1, 2, 8, 8)
    onnx_path = str(tmp_path / "m.onnx")
    ex.export(RoundTrip(), x, onnx_path)
    eng_path = str(tmp_path / "m.engine")
    assert cli.main(["--buildOnly", f"--onnx={onnx_path}", f"--saveEngine={eng_path}",
                     "--plugins=tensorrt_dft_plugins_amd/_C.so", "--device=cpu"]) == 0
    assert os.path.exists(eng_path)
    assert cli.main([f"--loadEngine={eng_path}", "--iterations=5", "--warmUp=1", "--device=cpu",
                     f"--exportTimes={tmp_path / 't.json'}"]) == 0
    out = capsys.readouterr().out
    assert "Throughput" in out and "Latency" in out


@pytest.mark.gpu
def test_engine_hipgraph_gpu(device, tmp_path):
    torch.manual_seed(0)
    x = torch.randn(2, 4, 720, 1440)
    eng = Engine.build(RoundTrip(), (x,), device=device)
    assert eng.use_graph and eng._cuda_graph is not None
    (z,) = eng.infer(x.to(device))
    assert torch.allclose(z.cpu(), 0.25 * x, atol=1e-5)
    p = str(tmp_path / "g.engine")
    eng.save(p)
    eng2 = Engine.load(p, device=device)
    xg = x.to(device)
    y = torch.empty(2, 4, 720, 1440, device=device)
    eng2.execute_v2([xg.data_ptr(), y.data_ptr()])
    assert torch.allclose(y.cpu(), 0.25 * x, atol=1e-5)
    st = eng2.benchmark(iterations=20, warmup=2)
    assert st["latency_median_ms"] > 0


@pytest.mark.gpu
def test_engine_from_fast_models_gpu(device, tmp_path):
    """Engines built from the MI355X model paths (com.amd.dft nodes) replay under hipGraph and
    match the eager model."""
    from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet, FNO2d, FNOConfig

    torch.manual_seed(0)
    fno = FNO2d(FNOConfig(img_size=(90, 180), modes1=12, modes2=12, n_layers=2), backend="amd").eval()
    x = torch.randn(2, 20, 90, 180)
    with torch.no_grad():
        ref = fno.to(device)(x.to(device))
    eng = Engine.build(fno.cpu(), (x,), device=device)
    assert eng.use_graph
    (y,) = eng.infer(x.to(device))
    assert torch.allclose(y, ref, atol=1e-4)

    cfg = AFNOConfig(img_size=(64, 128), in_chans=4, out_chans=4, embed_dim=64, depth=2, num_blocks=8)
    afno = AFNONet(cfg, backend="amd").eval()
    xa = torch.randn(1, 4, 64, 128)
    with torch.no_grad():
        refa = afno.to(device)(xa.to(device))
    p = str(tmp_path / "afno.engine")
    Engine.build(afno.cpu(), (xa,), device=device).save(p)
    (ya,) = Engine.load(p, device=device).infer(xa.to(device))
    assert torch.allclose(ya, refa, atol=1e-3)
