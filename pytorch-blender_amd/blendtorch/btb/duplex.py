"""Blender side of the bidirectional channel (reference: btb/duplex.py:8-67).

A PAIR socket that *binds*; HWM 10/10, send/receive timeouts (5 s default),
``recv(timeoutms)`` -> dict or None, ``send(**kw)`` adds ``btid`` and a random
32-bit ``btmid`` and returns the id.
"""
import os
import sys

from ..transport import zmq
from .constants import DEFAULT_TIMEOUTMS


class DuplexChannel:
    """Generic duplex messaging with a single PyTorch-side DuplexChannel."""

    def __init__(self, address, btid=None, lingerms=0, timeoutms=DEFAULT_TIMEOUTMS):
        self.ctx = zmq.Context()
        self.sock = self.ctx.socket(zmq.PAIR)
        self.sock.setsockopt(zmq.LINGER, lingerms)
        self.sock.setsockopt(zmq.RCVHWM, 10)
        self.sock.setsockopt(zmq.SNDHWM, 10)
        self.sock.setsockopt(zmq.SNDTIMEO, timeoutms)
        self.sock.setsockopt(zmq.RCVTIMEO, timeoutms)
        self.sock.bind(address)
        self.poller = zmq.Poller()
        self.poller.register(self.sock, zmq.POLLIN)
        self.btid = btid

    def recv(self, timeoutms=None):
        """Next message or None if nothing arrives within ``timeoutms``."""
        ready = dict(self.poller.poll(timeoutms))
        if self.sock in ready:
            return self.sock.recv_pyobj()
        return None

    def send(self, **kwargs):
        """Send ``kwargs`` with ``btid``/``btmid`` attached; returns ``btmid``."""
        mid = int.from_bytes(os.urandom(4), sys.byteorder)
        self.sock.send_pyobj({'btid': self.btid, 'btmid': mid, **kwargs})
        return mid

    def close(self):
        self.sock.close()
