import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running test")


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
