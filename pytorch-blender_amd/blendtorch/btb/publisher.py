"""Producer side of the data stream (reference: btb/publisher.py:4-43).

A PUSH socket that *binds* ``bind_address``: SNDHWM = ``send_hwm``,
LINGER = ``lingerms``, IMMEDIATE = 1 -- so ``publish`` blocks (backpressure)
while no consumer is connected or all consumer queues are full, and no
message is ever dropped.  Every message is the dict
``{'btid': btid, **kwargs}``, pickled.
"""
from ..transport import zmq


class DataPublisher:
    """Publish rendered images and auxiliary data to ``btt`` datasets."""

    def __init__(self, bind_address, btid=None, send_hwm=10, lingerms=0):
        self.ctx = zmq.Context()
        self.sock = self.ctx.socket(zmq.PUSH)
        self.sock.setsockopt(zmq.SNDHWM, send_hwm)
        self.sock.setsockopt(zmq.LINGER, lingerms)
        self.sock.setsockopt(zmq.IMMEDIATE, 1)
        self.sock.bind(bind_address)
        self.btid = btid

    def publish(self, **kwargs):
        """Send ``{'btid': btid, **kwargs}`` (values must be picklable)."""
        self.sock.send_pyobj({'btid': self.btid, **kwargs})

    def close(self):
        self.sock.close()
