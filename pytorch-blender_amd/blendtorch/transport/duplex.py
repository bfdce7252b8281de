"""PAIR-socket message channel shared by both ends of the duplex link.

The Blender side binds, and the PyTorch side connects to it (reference:
pkg_blender/blendtorch/btb/duplex.py:8-67, pkg_pytorch/blendtorch/btt/duplex.py:8-67).
Everything else is identical: 10-message high-water marks in both directions,
send/receive timeouts, ``recv`` that returns None when nothing arrives in time,
and ``send`` that stamps the sender's ``btid`` and a random 32-bit message id
``btmid`` onto the dict.
"""
import os

from . import zmq

HWM = 10


def _message_id():
    return int.from_bytes(os.urandom(4), 'little')


class PairChannel:
    def __init__(self, address, bind, btid=None, lingerms=0, timeoutms=10000):
        self.btid = btid
        self.ctx = zmq.Context()
        self.sock = self.ctx.socket(zmq.PAIR)
        for opt, val in ((zmq.LINGER, lingerms), (zmq.SNDHWM, HWM), (zmq.RCVHWM, HWM),
                         (zmq.SNDTIMEO, timeoutms), (zmq.RCVTIMEO, timeoutms)):
            self.sock.setsockopt(opt, val)
        (self.sock.bind if bind else self.sock.connect)(address)
        self.poller = zmq.Poller()
        self.poller.register(self.sock, zmq.POLLIN)

    def recv(self, timeoutms=None):
        """Next message dict, or None when nothing arrives within ``timeoutms``
        (None waits indefinitely)."""
        if self.sock in dict(self.poller.poll(timeoutms)):
            return self.sock.recv_pyobj()
        return None

    def send(self, **kwargs):
        """Send ``kwargs`` stamped with ``btid`` and a fresh ``btmid``; returns the id."""
        mid = _message_id()
        self.sock.send_pyobj({'btid': self.btid, 'btmid': mid, **kwargs})
        return mid

    def close(self):
        self.sock.close()
