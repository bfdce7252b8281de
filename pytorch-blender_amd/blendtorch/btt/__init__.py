"""PyTorch-side API of blendtorch (reference: pkg_pytorch/blendtorch/btt/__init__.py:1-8).

Public names match the reference: BlenderLauncher, LaunchInfo,
RemoteIterableDataset, FileDataset, discover_blender, FileRecorder,
FileReader, DuplexChannel, env.  MI355X additions: DeviceLoader and
DecodeConfig (``btt.gpu``, device-resident streaming) and DeviceReplayBuffer
(``btt.replay``, HBM-resident record/replay); imported lazily so the CPU API
works without the HIP extension.
"""
from .launcher import BlenderLauncher
from .launch_info import LaunchInfo
from .dataset import RemoteIterableDataset, FileDataset, SingleFileDataset
from .finder import discover_blender
from .file import FileRecorder, FileReader
from .duplex import DuplexChannel
from .utils import get_primary_ip
from .constants import DEFAULT_TIMEOUTMS
from . import env

__version__ = '0.2.0'


def __getattr__(name):
    if name in ('DeviceLoader', 'DecodeConfig'):
        from . import gpu
        return getattr(gpu, name)
    if name == 'DeviceReplayBuffer':
        from .replay import DeviceReplayBuffer
        return DeviceReplayBuffer
    raise AttributeError(name)
