"""GPU tier of the build-time graph optimizer: the reference's workflow at the benchmark sizes.

Stock contrib-exported FourCastNet (720x1440, embed 768, FourCastNet's 8 blocks of 96 channels)
and FNO2d (20 channels, 720x1440, 32x32 modes) -> ONNX -> engine built on the MI355X (rewrites
verified on the device) -> save -> load / ``dftexec --loadEngine``, compared against the plain
PyTorch fp32 models (/root/reference/tests/test_dft.py:124-184 is the tiny-grid original).
"""
import os
import subprocess
import sys

import pytest
import torch

from tensorrt_dft_plugins_amd.engine import Engine
from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet, FNO2d, FNOConfig
from tensorrt_dft_plugins_amd.onnx import exporter as ex

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


@pytest.fixture(scope="module")
def fcn_pair():
    torch.manual_seed(0)
    cfg = AFNOConfig(depth=2)
    m = AFNONet(cfg, backend="contrib").cuda().eval()
    ref = AFNONet(cfg, backend="torch").cuda().eval()
    ref.load_state_dict(m.state_dict())
    x = torch.randn(2, cfg.in_chans, *cfg.img_size, device="cuda")
    with torch.no_grad():
        want = ref(x)
    return cfg, m, x, want


def test_contrib_fourcastnet_engine_full_size(fcn_pair, tmp_path):
    cfg, m, x, want = fcn_pair
    from tensorrt_dft_plugins_amd.ops.spectral import fallback_counts, fallback_reset

    eng = Engine.build(m, (x,))
    opt = eng.header.extra["optimizer"]
    assert opt["applied"].get("afno_filter") == 2 and opt["applied"].get("layer_norm") == 4, opt
    assert opt["applied"].get("linear_gelu") == 2 and opt["applied"].get("linear_residual") == 2, opt
    assert opt["applied"].get("patch_embed") == 1 and opt["applied"].get("unpatch_head") == 1, opt
    assert opt["applied"].get("afno_block") == 2 and opt["applied"].get("afno_block_chain") == 1, opt
    assert opt["applied"].get("afno_block_head") == 1, opt
    assert not opt["rejected"], opt["rejected"]
    p = str(tmp_path / "fcn_contrib.engine")
    eng.save(p)
    eng2 = Engine.load(p)
    fallback_reset()
    (y,) = eng2.infer(x)
    torch.cuda.synchronize()
    err = _rel(y, want)
    print(f"contrib FourCastNet engine (depth 2, 720x1440) rel-L2 vs torch fp32: {err:.3e}")
    assert err < 5e-5
    assert not fallback_counts(), fallback_counts()  # every rewritten node ran its hand kernel


def test_contrib_fourcastnet_engine_unoptimized_matches(fcn_pair):
    cfg, m, x, want = fcn_pair
    eng = Engine.build(m, (x,), optimize=False)
    (y,) = eng.infer(x)
    assert _rel(y, want) < 1e-5


def test_contrib_fno_engine_full_size(tmp_path):
    torch.manual_seed(1)
    cfg = FNOConfig()  # 20 channels, 720x1440, 32x32 modes, 4 layers
    m = FNO2d(cfg, backend="contrib").cuda().eval()
    ref = FNO2d(cfg, backend="torch").cuda().eval()
    ref.load_state_dict(m.state_dict())
    x = torch.randn(1, cfg.in_chans, *cfg.img_size, device="cuda")
    with torch.no_grad():
        want = ref(x)
    onnx_path = str(tmp_path / "fno.onnx")
    ex.export(m, x, onnx_path)
    eng = Engine.build(onnx_path, shapes=[list(x.shape)])
    opt = eng.header.extra["optimizer"]
    assert opt["applied"].get("fno_spectral_pointwise_gelu") == 3 and opt["applied"].get("fno_spectral_pointwise") == 1
    (y,) = eng.infer(x)
    err = _rel(y, want)
    print(f"contrib FNO2d engine (720x1440) rel-L2 vs torch fp32: {err:.3e}")
    assert err < 1e-4
    # the saved engine through the trtexec-style CLI (reference README.md:71-75)
    eng_path = str(tmp_path / "fno.engine")
    eng.save(eng_path)
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-m", "tensorrt_dft_plugins_amd.engine.cli", f"--loadEngine={eng_path}",
                        "--plugins=tensorrt_dft_plugins_amd/_C.so", "--iterations=20", "--warmUp=3"],
                       capture_output=True, text=True, env=env, cwd=ROOT, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Throughput" in r.stdout
    print(r.stdout.strip().splitlines()[-1])


def test_contrib_fourcastnet_engine_headline_config():
    """The headline configuration through the reference's workflow: FourCastNet at depth 12,
    batch 32, 720x1440, written with the ONNX-contrib Rfft/Irfft + stock ops, exported, optimized (every block on the
    fused kernels, nothing rejected), serialized, deserialized and replayed -- against the torch fp32 model."""
    torch.manual_seed(2)
    cfg = AFNOConfig(depth=12)
    m = AFNONet(cfg, backend="contrib").cuda().eval()
    x = torch.randn(32, cfg.in_chans, *cfg.img_size, device="cuda")
    eng = Engine.build(m, (x,))
    opt = eng.header.extra["optimizer"]
    assert opt["applied"].get("afno_block") == 12 and not opt["rejected"], opt
    eng2 = Engine.deserialize(eng.serialize())
    del eng
    torch.cuda.empty_cache()
    (y,) = eng2.infer(x)
    del eng2
    torch.cuda.empty_cache()
    ref = AFNONet(cfg, backend="torch").cuda().eval()
    ref.load_state_dict(m.state_dict())
    with torch.no_grad():
        want = ref(x)
    err = _rel(y, want)
    print(f"contrib FourCastNet engine (depth 12, batch 32, 720x1440) rel-L2 vs torch fp32: {err:.3e}")
    assert err < 5e-5


def test_contrib_and_native_engines_agree():
    """The contrib-export engine (bench.py's headline) and the native-export engine run the same kernels: equal
    outputs to the last few bits at depth 2, batch 2, 720x1440 (profiles/engine_diff_r6.txt: same sequence at depth 12)."""
    torch.manual_seed(3)
    cfg = AFNOConfig(depth=2)
    x = torch.randn(2, cfg.in_chans, *cfg.img_size, device="cuda")
    outs, ops = {}, {}
    for backend in ("contrib", "amd"):
        torch.manual_seed(4)
        m = AFNONet(cfg, backend=backend).cuda().eval()
        eng = Engine.build(m, (x,))
        outs[backend] = eng.infer(x)[0]
        ops[backend] = [n[4] for n in eng.graph.nodes if n[4] != "Reshape"]
    assert ops["contrib"] == ops["amd"], ops
    assert _rel(outs["contrib"], outs["amd"]) < 1e-6
