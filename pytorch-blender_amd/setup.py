"""Packaging for blendtorch (MI355X).  Native parts are built in-tree by
``python -m blendtorch._build`` (g++ / hipcc --offload-arch=gfx950); the
package data below ships the resulting .so files and producer binaries."""
from setuptools import find_packages, setup

setup(
    name='blendtorch-mi355x',
    version='0.2.0',
    description='Stream Blender (or headless) renderings into PyTorch-ROCm on MI355X',
    packages=find_packages(include=['blendtorch', 'blendtorch.*']),
    package_data={'blendtorch': ['_native*.so', '_hip*.so', 'bin/*', 'btb/headless/bin/blender']},
    python_requires='>=3.7',
    install_requires=['numpy', 'torch'],
    entry_points={'console_scripts': ['blendtorch-launch=blendtorch.btt.apps.launch:main']},
)
