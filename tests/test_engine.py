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


def test_engine_execute_v2_copy_path_cpu():
    """No hipGraph on the CPU: caller buffers always go through the engine's bindings (counted)."""
    x = torch.randn(1, 1, 4, 8)
    eng = Engine.build(Rfft2Model(), (x,), device="cpu")
    y = torch.empty(1, 1, 4, 5, 2)
    for _ in range(3):
        assert eng.execute_v2([x, y])
    assert eng.bound_stats == {"copies": 3, "captures": 0, "replays": 0, "evictions": 0}
    assert torch.allclose(y, torch.view_as_real(torch.fft.rfft2(x)), atol=1e-5)


def test_engine_bound_graph_bookkeeping_cpu(monkeypatch):
    """The pointer-set bookkeeping of execute_async_v2 (bind on second use, LRU eviction, raw-pointer
    hot path, the engine's own buffers untouched) with a stand-in for the captured graph that runs
    the model eagerly on the bound views -- the GPU test covers the real capture."""
    x = torch.randn(1, 1, 4, 8)
    eng = Engine.build(Rfft2Model(), (x,), device="cpu")

    class FakeMain:  # "a main graph exists": replays the model on the engine's own buffers
        def replay(self):
            (o,) = eng.graph.run(eng.static_inputs[0])
            eng.static_outputs[0].copy_(o)

    eng._cuda_graph = FakeMain()

    class FakeGraph:
        def __init__(self, views):
            self.views, self.replays = views, 0

        def replay(self):
            self.replays += 1
            (o,) = eng.graph.run(self.views[0])
            self.views[1].copy_(o)

    monkeypatch.setattr(eng, "_capture_bound", lambda views: FakeGraph(views))
    eng.BOUND_GRAPH_MAX = 2
    bufs = [(torch.randn(1, 1, 4, 8), torch.empty(1, 1, 4, 5, 2)) for _ in range(3)]
    for _ in range(2):
        for xb, yb in bufs:
            assert eng.execute_async_v2([xb.data_ptr(), yb.data_ptr()])
            assert torch.allclose(yb, torch.view_as_real(torch.fft.rfft2(xb)), atol=1e-5)
    assert eng.bound_stats == {"copies": 3, "captures": 3, "replays": 3, "evictions": 1}
    assert len(eng._bound) == 2 and (bufs[0][0].data_ptr(), bufs[0][1].data_ptr()) not in eng._bound
    xb, yb = bufs[2]
    xb.copy_(torch.randn(1, 1, 4, 8))
    eng.execute_async_v2([xb.data_ptr(), yb.data_ptr()])  # hot path: raw pointers of a bound set
    assert eng.bound_stats["replays"] == 4
    assert torch.allclose(yb, torch.view_as_real(torch.fft.rfft2(xb)), atol=1e-5)
    eng.execute_async_v2([torch.randn(1, 1, 4, 8), torch.empty(1, 1, 4, 5, 4)[..., :2]])  # strided: copy path
    assert eng.bound_stats["copies"] == 4


def test_engine_execute_v2_own_bindings_zero_copy_cpu():
    """Bindings that are the engine's own buffers run in place (TensorRT-style preallocated
    bindings); execute_async_v2 returns without waiting."""
    x = torch.randn(1, 1, 4, 8)
    eng = Engine.build(Rfft2Model(), (x,), device="cpu")
    xin, yout = eng.binding_tensors
    xin.copy_(x)
    ptr_out = yout.data_ptr()
    assert eng.execute_v2(eng.binding_ptrs())
    assert yout.data_ptr() == ptr_out
    assert torch.allclose(yout, torch.view_as_real(torch.fft.rfft2(x)), atol=1e-5)
    y2 = torch.empty_like(yout)
    assert eng.execute_async_v2([xin.data_ptr(), y2.data_ptr()])  # mixed: own input, foreign output
    assert torch.allclose(y2, yout)


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
    # zero-copy: the engine's own bindings, graph replay straight on them
    eng2.binding_tensors[0].copy_(xg * 2)
    eng2.execute_v2(eng2.binding_ptrs())
    assert torch.allclose(eng2.binding_tensors[1].cpu(), 0.5 * x, atol=1e-5)
    st = eng2.benchmark(iterations=20, warmup=2)
    assert st["latency_median_ms"] > 0


@pytest.mark.gpu
def test_engine_execute_v2_bound_graphs_gpu(device):
    """Caller-owned device pointers: copied through the engine buffers on first use, then a graph
    captured on exactly those pointers (inputs read in place) is replayed; new data in the same
    buffers is picked up, LRU eviction past BOUND_GRAPH_MAX, results equal torch.fft throughout."""
    torch.manual_seed(3)
    eng = Engine.build(Rfft2Model(), (torch.randn(2, 3, 720, 1440),), device=device)
    eng.BOUND_GRAPH_MAX = 2
    bufs = [(torch.empty(2, 3, 720, 1440, device=device), torch.empty(2, 3, 720, 721, 2, device=device))
            for _ in range(3)]
    for rnd in range(3):
        for x, y in bufs:
            x.copy_(torch.randn(2, 3, 720, 1440))
            y.fill_(float("nan"))
            assert eng.execute_v2([x.data_ptr(), y.data_ptr()])
            ref = torch.view_as_real(torch.fft.rfft2(x.cpu().double()))
            err = ((y.cpu().double() - ref.double()).norm() / ref.double().norm()).item()
            assert err < 1e-6, (rnd, err)
    st = dict(eng.bound_stats)
    print("bound-graph stats", st)
    # round 0: 3 copies; round 1: 3 captures + replays (the third evicts buffer 0's graph); round 2:
    # buffer 0 is counted again (a copy), buffers 1 and 2 replay
    assert st == {"copies": 4, "captures": 3, "evictions": 1, "replays": 5}
    own_in, own_out = eng.binding_tensors
    own_in.copy_(bufs[0][0])
    eng.execute_v2(eng.binding_ptrs())  # the engine's own buffers: the main graph, no bookkeeping
    assert torch.equal(own_out, bufs[0][1]) and eng.bound_stats == st


@pytest.mark.gpu
def test_engine_execute_async_v2_inside_caller_capture_gpu(device):
    """execute_async_v2 on caller pointers while the CALLER is capturing a hipGraph: no nested
    capture / replay, the engine's nodes are recorded into the caller's graph."""
    torch.manual_seed(4)
    eng = Engine.build(Rfft2Model(), (torch.randn(1, 2, 720, 1440),), device=device)
    x = torch.randn(1, 2, 720, 1440, device=device)
    y = torch.empty(1, 2, 720, 721, 2, device=device)
    for _ in range(2):  # the same pointer set twice outside capture: bound graph, then replay
        eng.execute_async_v2([x.data_ptr(), y.data_ptr()])
    torch.cuda.synchronize()
    s = torch.cuda.Stream(device)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(g):
        eng.execute_async_v2([x.data_ptr(), y.data_ptr()])
    x.copy_(torch.randn(1, 2, 720, 1440))
    y.fill_(float("nan"))
    g.replay()
    torch.cuda.synchronize()
    ref = torch.view_as_real(torch.fft.rfft2(x.cpu().double()))
    assert ((y.cpu().double() - ref).norm() / ref.norm()).item() < 1e-6


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


class _Rfft2(nn.Module):
    def forward(self, x):
        return ex.OnnxRfft2.apply(x)


class _Irfft2(nn.Module):
    def forward(self, x):
        return ex.OnnxIrfft2.apply(x)


@pytest.mark.gpu
@pytest.mark.parametrize("op", ["rfft2", "irfft2"])
@pytest.mark.parametrize("dft_dim1", [1, 2])
@pytest.mark.parametrize("dft_dim2", [4])
@pytest.mark.parametrize("num_c", [1, 3])
@pytest.mark.parametrize("batch_size", [1, 2])
def test_reference_grid_through_engine_gpu(device, tmp_path, op, dft_dim1, dft_dim2, num_c, batch_size):
    """The reference's 16 cases (/root/reference/tests/test_dft.py:124-184) on the GPU through
    export -> Engine.build (hipGraph) -> save -> load -> execute_v2(device pointers)."""
    torch.manual_seed(1)
    x = torch.randn(batch_size, num_c, dft_dim1, dft_dim2)
    if op == "rfft2":
        model, inp = _Rfft2(), x
        expected = torch.view_as_real(torch.fft.rfft2(x, dim=(-2, -1), norm="backward"))
    else:
        inp = torch.view_as_real(torch.fft.rfft2(x))
        model = _Irfft2()
        expected = torch.fft.irfft2(torch.view_as_complex(inp), dim=(-2, -1))
    p = str(tmp_path / f"{op}.engine")
    Engine.build(model, (inp,), device=device).save(p)
    eng = Engine.load(p, device=device)
    assert eng.use_graph and eng._cuda_graph is not None
    xin = inp.to(device)
    out = torch.empty(eng.bindings[-1].shape, device=device)
    assert eng.execute_v2([xin.data_ptr(), out.data_ptr()])
    assert torch.allclose(out.cpu(), expected, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fourcastnet_full_grid_engine_gpu(device, tmp_path, dtype):
    """FourCastNet at the full 720x1440 grid (depth 2) exported with its com.amd.dft nodes,
    saved, loaded and replayed from the engine file: matches the captured module."""
    from tensorrt_dft_plugins_amd.engine.capture import CapturedModule
    from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet
    from helpers import rel_l2

    torch.manual_seed(3)
    m = AFNONet(AFNOConfig(depth=2), backend="amd").to(device).to(dtype).eval()
    x = torch.randn(2, 20, 720, 1440, device=device).to(dtype)
    (ref,) = CapturedModule(m, [x]).replay()
    p = str(tmp_path / "fcn.engine")
    Engine.build(m, (x,), device=device).save(p)
    eng = Engine.load(p, device=device)
    (y,) = eng.infer(x)
    assert y.dtype == dtype and y.shape == ref.shape
    assert rel_l2(y.float(), ref.float()) < (1e-5 if dtype == torch.float32 else 1e-2)
