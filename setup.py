"""pip install -e .  ->  builds the native library in-tree (gfx950) and installs the package.

Mirrors the reference's setup.py-drives-the-native-build arrangement
(/root/reference/setup.py:30-48), without its fragile path arithmetic: the build step is
``tensorrt_dft_plugins_amd._build`` (hipcc, incremental), or CMake when MI_DFT_USE_CMAKE=1.
"""
import os
import subprocess
import sys

from setuptools import Extension, setup
from setuptools.command.build_ext import build_ext

ROOT = os.path.dirname(os.path.abspath(__file__))


class NativeBuild(build_ext):
    def run(self):
        if os.environ.get("MI_DFT_USE_CMAKE") == "1":
            bdir = os.path.join(ROOT, "build", "cmake")
            subprocess.check_call(["cmake", "-S", ROOT, "-B", bdir, "-G", "Ninja"])
            subprocess.check_call(["cmake", "--build", bdir, "-j", str(os.cpu_count() or 8)])
        else:
            subprocess.check_call([sys.executable, "-m", "tensorrt_dft_plugins_amd._build"], cwd=ROOT)


setup(ext_modules=[Extension("tensorrt_dft_plugins_amd._C", sources=[])], cmdclass={"build_ext": NativeBuild})
