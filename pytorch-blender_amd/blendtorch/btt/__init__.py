"""PyTorch-side API of blendtorch (reference: pkg_pytorch/blendtorch/btt/__init__.py:1-8).

Public names match the reference: BlenderLauncher, LaunchInfo,
RemoteIterableDataset, FileDataset, discover_blender, FileRecorder,
FileReader, DuplexChannel, env.  MI355X additions: DeviceLoader and
DecodeConfig (``btt.gpu``), the device-resident streaming path.
"""
from .launcher import BlenderLauncher
from .launch_info import LaunchInfo
from .finder import discover_blender
from .utils import get_primary_ip
from .constants import DEFAULT_TIMEOUTMS

__version__ = '0.2.0'


def __getattr__(name):
    # heavy / optional pieces import lazily (torch, HIP extension)
    if name in ('DeviceLoader', 'DecodeConfig'):
        from . import gpu
        return getattr(gpu, name)
    raise AttributeError(name)
