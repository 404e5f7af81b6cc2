"""Observability: opt-in roctx op ranges, Python trace ranges, logger."""
import logging
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_ops_run_with_native_tracing_enabled():
    """MI_DFT_TRACE=1 wraps every op in a roctx range (dlopen'ed): results must be unchanged."""
    code = "\n".join([
        "import torch, tensorrt_dft_plugins_amd as t",
        "t.load_plugins()",
        "from tensorrt_dft_plugins_amd.utils.trace import trace_range",
        "x = torch.randn(2, 6, 16)",
        "with trace_range('test.range'):",
        "    y = torch.ops.amd_dft.r2c(x, [1, 2], 1.0)",
        "ref = torch.view_as_real(torch.fft.rfft2(x))",
        "assert torch.allclose(y, ref, atol=1e-4), (y - ref).abs().max()",
        "print('ok')",
    ])
    env = dict(os.environ, MI_DFT_TRACE="1", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "ok" in r.stdout


def test_trace_range_is_noop_when_disabled(monkeypatch):
    from tensorrt_dft_plugins_amd.utils.trace import trace_range, tracing_enabled

    monkeypatch.delenv("MI_DFT_TRACE", raising=False)
    assert not tracing_enabled()
    with trace_range("nothing"):
        pass


def test_logger_level_from_env():
    code = ("from tensorrt_dft_plugins_amd.utils.trace import get_logger;"
            "import logging; print(get_logger('engine').getEffectiveLevel())")
    env = dict(os.environ, MI_DFT_LOG="debug", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert int(r.stdout.strip()) == logging.DEBUG
