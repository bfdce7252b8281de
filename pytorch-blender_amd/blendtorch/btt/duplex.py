"""PyTorch end of the duplex link to one producer instance: connects to the
address the instance bound (10 s default timeouts; ``btid`` is None on this
side). Protocol in :mod:`blendtorch.transport.duplex`."""
from ..transport.duplex import PairChannel
from .constants import DEFAULT_TIMEOUTMS


class DuplexChannel(PairChannel):
    """Messages to and from a Blender-side ``btb.DuplexChannel``."""

    def __init__(self, address, btid=None, lingerms=0, timeoutms=DEFAULT_TIMEOUTMS):
        super().__init__(address, bind=False, btid=btid, lingerms=lingerms, timeoutms=timeoutms)
