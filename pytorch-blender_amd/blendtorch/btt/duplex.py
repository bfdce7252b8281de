"""Bidirectional channel to one producer instance (PyTorch side).

Reference: pkg_pytorch/blendtorch/btt/duplex.py:8-67 -- a PAIR socket that
*connects* (the Blender side binds), HWM 10/10, send/receive timeouts,
``recv(timeoutms)`` returning None on silence, and ``send(**kw)`` adding
``btid`` (None on this side) and a random 32-bit message id ``btmid``.
"""
import os
import sys

from ..transport import zmq
from .constants import DEFAULT_TIMEOUTMS


class DuplexChannel:
    """Generic duplex messaging with a remote (Blender-side) DuplexChannel."""

    def __init__(self, address, btid=None, lingerms=0, timeoutms=DEFAULT_TIMEOUTMS):
        self.ctx = zmq.Context()
        self.sock = self.ctx.socket(zmq.PAIR)
        self.sock.setsockopt(zmq.LINGER, lingerms)
        self.sock.setsockopt(zmq.RCVHWM, 10)
        self.sock.setsockopt(zmq.SNDHWM, 10)
        self.sock.setsockopt(zmq.SNDTIMEO, timeoutms)
        self.sock.setsockopt(zmq.RCVTIMEO, timeoutms)
        self.sock.connect(address)
        self.poller = zmq.Poller()
        self.poller.register(self.sock, zmq.POLLIN)
        self.btid = btid

    def recv(self, timeoutms=None):
        """Next message (dict) or None when nothing arrives within ``timeoutms``
        (None blocks until a message is available)."""
        ready = dict(self.poller.poll(timeoutms))
        if self.sock in ready:
            return self.sock.recv_pyobj()
        return None

    def send(self, **kwargs):
        """Send ``kwargs`` plus ``btid`` and a fresh ``btmid``; returns the id."""
        mid = int.from_bytes(os.urandom(4), sys.byteorder)
        self.sock.send_pyobj({'btid': self.btid, 'btmid': mid, **kwargs})
        return mid

    def close(self):
        self.sock.close()
