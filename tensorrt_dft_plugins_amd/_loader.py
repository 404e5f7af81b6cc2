"""Native library loading and the plugin registry.

Parity with the reference's ``trt_dft_plugins.load_plugins()``
(/root/reference/src/trt_dft_plugins/__init__.py:26-32), which ``dlopen``s
``libtrt_dft_plugins.so`` from the package directory so that its static registrars put the
``Rfft``/``Irfft`` creators into TensorRT's global registry.  Here the library is
``_C.so`` next to this file and its static ``TORCH_LIBRARY`` initialisers register the
``torch.ops.amd_dft`` operators (``Rfft``, ``Irfft``, ``r2c``, ``c2r``, ``c2c`` and the
spectral-layer kernels) with the PyTorch dispatcher.
"""
from __future__ import annotations

import json
import os
import threading

import torch

_LIB_PATH = os.environ.get("MI_DFT_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_C.so")
_lock = threading.Lock()
_loaded = False


class NativeLibraryMissing(RuntimeError):
    pass


def native_library_path() -> str:
    return _LIB_PATH


def load_plugins() -> None:
    """Load the native op library (idempotent).  Same name and signature as the reference.

    Raises ``NativeLibraryMissing`` when ``_C.so`` has not been built: there is no silent
    fallback, so a GPU run can never pass on an eager/PyTorch path by accident.
    """
    global _loaded
    if _loaded:
        return
    with _lock:
        if _loaded:
            return
        if not os.path.exists(_LIB_PATH):
            raise NativeLibraryMissing(
                f"{_LIB_PATH} not found: build it with `python -m tensorrt_dft_plugins_amd._build` "
                "(or `python setup.py build_ext --inplace`)")
        torch.ops.load_library(_LIB_PATH)
        _loaded = True


def is_loaded() -> bool:
    return _loaded


def build_info() -> str:
    """Provenance of the loaded library: ``amd_dft_source_digest=<sha256 of csrc/> host=<builder>
    time=<UTC>`` (embedded at link time by ``_build``)."""
    import ctypes

    load_plugins()
    fn = getattr(ctypes.CDLL(_LIB_PATH), "amd_dft_build_info", None)
    if fn is None:  # an older / diagnostic library (MI_DFT_LIB) without the provenance symbol
        return "unknown (no provenance symbol)"
    fn.restype = ctypes.c_char_p
    return fn().decode()


def plugin_registry() -> list[dict]:
    """Registered plugin creators: name, version, namespace, ONNX domain and attribute fields.

    Mirrors ``trt.get_plugin_registry().plugin_creator_list`` used by the reference's
    ``test_plugins_load`` (/root/reference/tests/test_dft.py:118-121).
    """
    load_plugins()
    return json.loads(torch.ops.amd_dft.plugin_registry())


def plugin_names() -> set[str]:
    return {p["name"] for p in plugin_registry()}


def get_plugin_creator(name: str, version: str = "1", namespace: str = "") -> dict:
    for p in plugin_registry():
        if p["name"] == name and p["version"] == version and p["namespace"] == namespace:
            return p
    raise KeyError(f"no plugin creator {name!r} version {version!r} in namespace {namespace!r}")
