"""Blender end of the duplex link: binds ``address`` (5 s default timeouts).
Protocol in :mod:`blendtorch.transport.duplex`."""
from ..transport.duplex import PairChannel
from .constants import DEFAULT_TIMEOUTMS


class DuplexChannel(PairChannel):
    """Messages to and from the PyTorch-side ``btt.DuplexChannel``."""

    def __init__(self, address, btid=None, lingerms=0, timeoutms=DEFAULT_TIMEOUTMS):
        super().__init__(address, bind=True, btid=btid, lingerms=lingerms, timeoutms=timeoutms)
