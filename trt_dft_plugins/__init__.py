"""Drop-in name of the reference package (``from trt_dft_plugins import load_plugins``).

The reference exposes exactly one function, ``load_plugins()``
(/root/reference/src/trt_dft_plugins/__init__.py:26-32); this module re-exports the
MI355X-native implementation from :mod:`tensorrt_dft_plugins_amd`.
"""
from tensorrt_dft_plugins_amd import load_plugins, plugin_names, plugin_registry  # noqa: F401
