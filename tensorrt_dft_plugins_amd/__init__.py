"""tensorrt_dft_plugins_amd -- MI355X-native DFT inference-op library.

Same capabilities as DistributedSpectrum/tensorrt-dft-plugins (``load_plugins()``, the
ONNX-contrib ``com.microsoft::Rfft`` / ``Irfft`` operators, export -> engine -> run), built
for AMD Instinct MI355X (gfx950): hand-written HIP Stockham FFT kernels registered as
PyTorch-ROCm custom ops, MFMA spectral-layer kernels, hipGraph engines and RCCL
data-parallel inference.
"""
from ._loader import (  # noqa: F401
    NativeLibraryMissing, build_info, get_plugin_creator, is_loaded, load_plugins, native_library_path, plugin_names,
    plugin_registry,
)
from .ops.dft import (  # noqa: F401
    contrib_irfft, contrib_rfft, fft, fftn, ifft, ifftn, irfft, irfft2, irfftn, rfft, rfft2, rfftn,
)

__version__ = "1.0.0"
PLUGIN_VERSION = "1"
