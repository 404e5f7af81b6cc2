import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


_BOX_BUILD = {}


def _gpu_tier(config) -> bool:
    expr = (config.option.markexpr or "").replace(" ", "")
    return "gpu" in expr and "notgpu" not in expr


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running test")
    # GPU tier on a GPU box: compile the native library from source HERE before any test loads it
    # (every object compiled on this host, the in-tree _C.so relinked; the reference builds then
    # tests in one command, /root/reference/build_with_docker.sh:39).  device_count() does not
    # initialise HIP.  MI_DFT_BOX_BUILD=0 skips it (the pushed library is then checked by digest).
    if _gpu_tier(config) and torch.cuda.device_count() > 0 and not os.environ.get("MI_DFT_LIB") \
            and os.environ.get("MI_DFT_BOX_BUILD", "1") != "0":
        import time

        from tensorrt_dft_plugins_amd import _build

        t0 = time.time()
        try:
            _build.build(from_source=True, verbose=True)
            _BOX_BUILD["seconds"] = time.time() - t0
        except Exception as e:  # keep the tier runnable on the pushed library, and say so loudly
            _BOX_BUILD["error"] = str(e).splitlines()[0] if str(e) else type(e).__name__
            print(f"[amd_dft build] FROM-SOURCE BUILD ON THIS HOST FAILED: {e}", flush=True)


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    if not _gpu_tier(config):
        return
    from tensorrt_dft_plugins_amd import _build, _loader

    st = _build.library_status(_loader.native_library_path())
    line = f"native library {st['path']}: source digest {'matches' if st['digest_ok'] else 'DOES NOT MATCH'} csrc/"
    if "error" in _BOX_BUILD:
        line += f"; the from-source build on this host FAILED ({_BOX_BUILD['error']}), the pushed library ran"
    if "seconds" in _BOX_BUILD:
        line += f"; compiled from source on this host before the tests ({_BOX_BUILD['seconds']:.0f} s)"
    if _loader.is_loaded():
        line += f"; loaded: {_loader.build_info()}"
    terminalreporter.write_line(line)


@pytest.fixture(scope="session", autouse=True)
def load_native_plugins():
    """Session-scoped, autouse: load the op library once (reference: tests/test_dft.py:63-65)."""
    from tensorrt_dft_plugins_amd import load_plugins

    load_plugins()


@pytest.fixture()
def device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU in this environment")
    return torch.device("cuda:0")
