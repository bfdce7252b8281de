"""Blender-side API of blendtorch (reference: pkg_blender/blendtorch/btb/__init__.py:1-9).

Runs inside Blender's Python.  Outside Blender (no ``bpy``), the headless
emulation in :mod:`blendtorch.btb.headless` is installed first, so producer
scripts -- and this package -- run unmodified in plain Python as well.
"""
import logging as _logging

try:
    import bpy as _bpy  # noqa: F401
except ImportError:
    from . import headless as _headless
    _headless.install()
    _logging.getLogger('blendtorch').info('bpy not found: using the headless Blender emulation')

from .animation import AnimationController
from .offscreen import OffScreenRenderer
from .arguments import parse_blendtorch_args
from .publisher import DataPublisher
from .camera import Camera
from .duplex import DuplexChannel
from .signal import Signal
from . import env, utils

__version__ = '0.2.0'
