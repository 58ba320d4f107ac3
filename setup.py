"""Packaging for ``imaginaire_amd`` (reference scripts/install.sh:38-51 builds its CUDA
extensions with per-extension setup.py files; here one in-tree gfx950 HIP extension).

    pip install -e . --no-build-isolation     # or: python setup.py develop
    python setup.py build_ext --inplace       # just the extension (imaginaire_amd/_C.so)
"""
import os
import subprocess
import sys

from setuptools import find_packages, setup
from setuptools.command.build_ext import build_ext
from setuptools.extension import Extension

HERE = os.path.dirname(os.path.abspath(__file__))


class HipBuild(build_ext):
    """Delegate to imaginaire_amd._build (hipcc --offload-arch=gfx950, parallel, cached)."""

    def run(self):
        subprocess.check_call([sys.executable, '-m', 'imaginaire_amd._build'], cwd=HERE)
        if not self.inplace:
            dst = os.path.join(self.build_lib, 'imaginaire_amd')
            os.makedirs(dst, exist_ok=True)
            self.copy_file(os.path.join(HERE, 'imaginaire_amd', '_C.so'),
                           os.path.join(dst, '_C.so'))


setup(
    name='imaginaire_amd',
    version='0.1.0',
    description='MI355X-native conditional image/video GAN framework (Imaginaire capabilities)',
    packages=find_packages(include=['imaginaire_amd', 'imaginaire_amd.*']),
    package_data={'imaginaire_amd': ['csrc/*.hip', 'csrc/*.cpp', 'csrc/*.h', '_C.so']},
    ext_modules=[Extension('imaginaire_amd._C', sources=[])],
    cmdclass={'build_ext': HipBuild},
    python_requires='>=3.8',
    install_requires=['torch', 'numpy', 'scipy', 'pyyaml', 'pillow'],
)
