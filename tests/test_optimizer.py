"""Build-time graph optimizer (onnx/optimizer.py): the reference's workflow -- a stock model whose
FFTs are the ONNX-contrib Rfft / Irfft functions (/root/reference/tests/test_dft.py:35-60), exported
to ONNX (:73-86), built into an engine (:89-101) and run (:104-115) -- with the engine build mapping
the spectral, LayerNorm and MLP patterns onto this library's kernels.

CPU tier: the rewrites run against the ops' CPU implementations (ATen references of the same
kernels), so these tests pin the pattern matching, the numeric identification and the rewritten
graph's semantics; the GPU tier (``test_optimizer_gpu``) repeats them at the benchmark sizes on the
hand kernels.
"""
import json
import os
import subprocess
import sys

import pytest
import torch
import torch.nn as nn

from tensorrt_dft_plugins_amd.engine import Engine
from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet, FNO2d, FNOConfig
from tensorrt_dft_plugins_amd.onnx import exporter as ex
from tensorrt_dft_plugins_amd.onnx import proto as P
from tensorrt_dft_plugins_amd.onnx.optimizer import optimize
from tensorrt_dft_plugins_amd.onnx.runner import OnnxGraph

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# smallest FourCastNet-shaped net whose every pattern has a kernel: H = 64 tokens (fused AFNO
# H-filter), block size 64, GEMM widths in 256-tiles, patch 8
SMALL_AFNO = dict(img_size=(512, 1024), in_chans=4, out_chans=4, embed_dim=256, depth=2, num_blocks=4, patch_size=8)


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


def _afno_pair(seed=0, **kw):
    torch.manual_seed(seed)
    cfg = AFNOConfig(**dict(SMALL_AFNO, **kw))
    m = AFNONet(cfg, backend="contrib").eval()
    ref = AFNONet(cfg, backend="torch").eval()
    ref.load_state_dict(m.state_dict())
    return cfg, m, ref


def _ops(data):
    return [(n.domain, n.op_type) for n in P.load_model(data).graph.node]


def test_contrib_models_match_torch_backend():
    cfg, m, ref = _afno_pair(depth=1)
    x = torch.randn(1, 4, *cfg.img_size)
    with torch.no_grad():
        assert _rel(m(x), ref(x)) < 1e-5
    torch.manual_seed(1)
    fcfg = FNOConfig(img_size=(32, 48), in_chans=3, out_chans=2, width=8, modes1=4, modes2=5, n_layers=2, proj_hidden=16)
    f = FNO2d(fcfg, backend="contrib").eval()
    fr = FNO2d(fcfg, backend="torch").eval()
    fr.load_state_dict(f.state_dict())
    xf = torch.randn(2, 3, 32, 48)
    with torch.no_grad():
        assert _rel(f(xf), fr(xf)) < 1e-5


def test_contrib_fourcastnet_exports_stock_graph():
    cfg, m, _ = _afno_pair(depth=1)
    data = ex.export(m, torch.randn(1, 4, *cfg.img_size))
    ops = _ops(data)
    assert ("com.microsoft", "Rfft") in ops and ("com.microsoft", "Irfft") in ops
    assert not any(d == "com.amd.dft" for d, _ in ops)  # nothing library-private in the stock export
    assert ("", "Einsum") in ops and ("", "MatMul") in ops and ("", "Erf") in ops


def test_optimizer_rewrites_contrib_fourcastnet():
    cfg, m, ref = _afno_pair()
    x = torch.randn(1, 4, *cfg.img_size)
    with torch.no_grad():
        want = ref(x)
    data = ex.export(m, x)
    od, rep = optimize(data, [list(x.shape)], [x.dtype], device="cpu")
    assert not rep.rejected, rep.rejected
    assert rep.count("afno_filter") == 2 and rep.count("layer_norm") == 4
    assert rep.count("linear_gelu") == 2 and rep.count("linear_residual") == 2
    assert rep.count("patch_embed") == 1 and rep.count("unpatch_head") == 1
    assert rep.count("split_fused_layer_norm_split") == 2 and rep.count("split_fused_linear3") == 2
    # both AFNO skips (filter input and block residual) fused into the C2R store
    assert all(a["skips"] == 2 for a in rep.applied if a["pattern"] == "afno_filter")
    # whole blocks in the native fp32 sequence: LN1 inside the W-transform, both skips + fc1's split
    # pairs + LN2 partials in the C2R epilogue, LN2 folded into fc1, LN1 statistics from fc2
    assert rep.count("afno_block") == 2 and rep.count("afno_block_chain") == 1 and rep.count("afno_block_head") == 1
    ops = [o for d, o in _ops(od)]
    assert "Rfft" not in ops and "Einsum" not in ops and "MatMul" not in ops
    assert ops.count("afno_spectral") == 2 and ops.count("r2c_ln") == 2 and ops.count("c2r_ln_add_split") == 2
    assert ops.count("linear3_ln") == 2 and ops.count("linear3_stats") == 1 and ops.count("linear3") == 1
    assert "layer_norm" not in ops and "layer_norm_split" not in ops and "split_bf16" not in ops
    assert rep.nodes_after < rep.nodes_before // 5
    (y,) = OnnxGraph(od, device="cpu").run(x)
    assert _rel(y, want) < 2e-5


def test_optimizer_rewrites_contrib_fno():
    torch.manual_seed(2)
    cfg = FNOConfig(img_size=(32, 48), in_chans=3, out_chans=2, width=8, modes1=4, modes2=5, n_layers=3, proj_hidden=16)
    m = FNO2d(cfg, backend="contrib").eval()
    ref = FNO2d(cfg, backend="torch").eval()
    ref.load_state_dict(m.state_dict())
    x = torch.randn(2, 3, 32, 48)
    with torch.no_grad():
        want = ref(x)
    od, rep = optimize(ex.export(m, x), [list(x.shape)], [x.dtype], device="cpu")
    assert not rep.rejected, rep.rejected
    assert rep.count("fno_spectral_pointwise_gelu") == 2 and rep.count("fno_spectral_pointwise") == 1
    assert rep.count("pointwise_conv") == 2 and rep.count("pointwise_conv_gelu") == 1
    assert all(a["modes"] == [4, 5] for a in rep.applied if a["pattern"].startswith("fno_spectral"))
    ops = [o for _, o in _ops(od)]
    assert ops.count("fno_mix_c2c") == 3 and ops.count("fno_c2r_pw") == 3 and "Irfft" not in ops
    (y,) = OnnxGraph(od, device="cpu").run(x)
    assert _rel(y, want) < 1e-5


class _OddMixing(nn.Module):
    """A spectral layer whose kept modes are NOT an FNO window (every other W mode): the
    optimizer must identify that and keep the stock nodes."""

    def __init__(self):
        super().__init__()
        self.w = nn.Parameter(torch.randn(3, 3) * 0.3)

    def forward(self, x):
        X = ex.OnnxRfft2.apply(x)  # [B, C, H, wf, 2]
        Y = torch.einsum("bihwk,io->bohwk", X, self.w)
        mask = torch.zeros(1, 1, 1, X.shape[3], 1)
        mask[..., ::2, :] = 1.0
        return ex.OnnxIrfft2.apply(Y * mask)


def test_optimizer_keeps_unrecognised_spectral_region():
    torch.manual_seed(3)
    m = _OddMixing().eval()
    x = torch.randn(2, 3, 16, 24)
    with torch.no_grad():
        want = m(x)
    od, rep = optimize(ex.export(m, x), [list(x.shape)], [x.dtype], device="cpu")
    assert not any(a["pattern"].startswith("fno_spectral") for a in rep.applied)
    assert any(r["pattern"] == "fno_spectral" and "window" in r["why"] for r in rep.rejected), rep.rejected
    (y,) = OnnxGraph(od, device="cpu").run(x)
    assert _rel(y, want) < 1e-6


def test_optimizer_verification_rejects_a_wrong_rewrite(monkeypatch):
    """Every rewrite is checked numerically against the nodes it replaces: a deliberately wrong
    replacement (GELU dropped from the fused GEMM) is refused and the stock nodes stay."""
    from tensorrt_dft_plugins_amd.onnx import optimizer as O

    class M(nn.Module):
        def __init__(self):
            super().__init__()
            self.fc = nn.Linear(128, 256)

        def forward(self, x):
            return torch.nn.functional.gelu(self.fc(x))

    torch.manual_seed(4)
    m = M().eval()
    x = torch.randn(4, 128)
    real = O.amd_node

    def broken(g, opname, tensors, outputs, **kw):
        if opname == "linear3":
            kw["act"] = 0
        return real(g, opname, tensors, outputs, **kw)

    monkeypatch.setattr(O, "amd_node", broken)
    od, rep = optimize(ex.export(m, x), [list(x.shape)], [x.dtype], device="cpu")
    assert not any(a["pattern"].startswith("linear") for a in rep.applied)
    assert any("verification failed" in r["why"] for r in rep.rejected)
    with torch.no_grad():
        want = m(x)
    (y,) = OnnxGraph(od, device="cpu").run(x)
    assert _rel(y, want) < 1e-6


def test_engine_build_optimizes_and_records_report(tmp_path):
    cfg, m, ref = _afno_pair(depth=1)
    x = torch.randn(1, 4, *cfg.img_size)
    data = ex.export(m, x)
    eng = Engine.build(data, shapes=[list(x.shape)], device="cpu")
    opt = eng.header.extra["optimizer"]
    assert opt["applied"]["afno_filter"] == 1 and opt["nodes_after"] < opt["nodes_before"]
    p = str(tmp_path / "fcn.engine")
    eng.save(p)
    eng2 = Engine.load(p, device="cpu")  # the saved engine holds the rewritten graph: no re-optimisation
    assert not hasattr(eng2, "optimize_report")
    assert any(n[4] == "afno_spectral" for n in eng2.graph.nodes)
    with torch.no_grad():
        want = ref(x)
    (y,) = eng2.infer(x)
    assert _rel(y, want) < 2e-5
    plain = Engine.build(data, shapes=[list(x.shape)], device="cpu", optimize=False)
    assert "optimizer" not in plain.header.extra
    assert _rel(plain.infer(x)[0], want) < 1e-5


def test_dftexec_builds_and_loads_contrib_fno(tmp_path):
    torch.manual_seed(5)
    cfg = FNOConfig(img_size=(32, 48), in_chans=3, out_chans=2, width=8, modes1=4, modes2=5, n_layers=2, proj_hidden=16)
    m = FNO2d(cfg, backend="contrib").eval()
    x = torch.randn(1, 3, 32, 48)
    onnx_path, eng_path = str(tmp_path / "fno.onnx"), str(tmp_path / "fno.engine")
    ex.export(m, x, onnx_path)
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    cli = [sys.executable, "-m", "tensorrt_dft_plugins_amd.engine.cli", "--device=cpu"]
    r = subprocess.run(cli + ["--buildOnly", f"--onnx={onnx_path}", f"--saveEngine={eng_path}",
                              "--plugins=tensorrt_dft_plugins_amd/_C.so"], capture_output=True, text=True, env=env,
                       cwd=ROOT, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "graph optimizer" in r.stdout and "fno_spectral" in r.stdout
    times = str(tmp_path / "t.json")
    r = subprocess.run(cli + [f"--loadEngine={eng_path}", "--iterations=3", "--warmUp=1", f"--exportTimes={times}"],
                       capture_output=True, text=True, env=env, cwd=ROOT, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.load(open(times))["iterations"] == 3


def test_optimizer_grouped_patch_conv_keeps_stock_nodes():
    """A grouped k = stride = 8 convolution is not the patch embedding: the rewrite is rejected with
    a reason and the build keeps the stock Conv, whose result is unchanged."""

    class M(nn.Module):
        def __init__(self):
            super().__init__()
            self.pe = nn.Conv2d(4, 64, kernel_size=8, stride=8, groups=2)

        def forward(self, x):
            return self.pe(x).flatten(2).transpose(1, 2)

    torch.manual_seed(6)
    m = M().eval()
    x = torch.randn(1, 4, 16, 32)
    od, rep = optimize(ex.export(m, x), [list(x.shape)], [x.dtype], device="cpu")
    assert not any(a["pattern"] == "patch_embed" for a in rep.applied)
    assert any(r["pattern"] == "patch_embed" and "group" in r["why"] for r in rep.rejected), rep.rejected
    with torch.no_grad():
        want = m(x)
    (y,) = OnnxGraph(od, device="cpu").run(x)
    assert _rel(y, want) < 1e-6


def test_optimizer_unexpected_error_rejects_instead_of_failing(monkeypatch):
    """Any exception inside a rewrite (not only RewriteRejected) drops that rewrite with its reason
    and the build goes on with the original nodes (a TypeError / KeyError / TORCH_CHECK
    used to abort the whole engine build)."""
    from tensorrt_dft_plugins_amd.onnx import optimizer as O

    class M(nn.Module):
        def __init__(self):
            super().__init__()
            self.fc = nn.Linear(128, 256)

        def forward(self, x):
            return torch.nn.functional.gelu(self.fc(x))

    torch.manual_seed(7)
    m = M().eval()
    x = torch.randn(4, 128)

    def boom(*a, **k):
        raise KeyError("simulated missing constant")

    monkeypatch.setattr(O, "_verify", boom)
    od, rep = optimize(ex.export(m, x), [list(x.shape)], [x.dtype], device="cpu")
    assert not rep.applied
    assert any("KeyError" in r["why"] for r in rep.rejected), rep.rejected
    with torch.no_grad():
        want = m(x)
    (y,) = OnnxGraph(od, device="cpu").run(x)
    assert _rel(y, want) < 1e-6
