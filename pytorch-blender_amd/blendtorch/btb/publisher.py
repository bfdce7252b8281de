"""Producer side of the data stream (reference: btb/publisher.py:4-43).

A PUSH socket that *binds* ``bind_address``: SNDHWM = ``send_hwm``,
LINGER = ``lingerms``, IMMEDIATE = 1 -- so ``publish`` blocks (backpressure)
while no consumer is connected or all consumer queues are full, and no
message is ever dropped.  Every message is the dict
``{'btid': btid, **kwargs}``, pickled.
"""
import os

import numpy as np

from ..transport import shm, zmq


class DataPublisher:
    """Publish rendered images and auxiliary data to ``btt`` datasets.

    ``shm_slots > 0`` (same-host consumers only): u8 ndarrays under
    ``shm_key`` travel through an N-slot shared-memory ring and the message
    carries a small descriptor instead of the pixels.  ``None`` (default)
    takes the value from ``BLENDTORCH_SHM_SLOTS`` (set by
    ``btt.BlenderLauncher(shm_slots=N)``), else 0: plain pickled frames as
    in the reference.
    """

    def __init__(self, bind_address, btid=None, send_hwm=10, lingerms=0, shm_slots=None, shm_key='image'):
        if shm_slots is None:
            shm_slots = int(os.environ.get('BLENDTORCH_SHM_SLOTS', '0') or 0)
        self.ctx = zmq.Context()
        self.sock = self.ctx.socket(zmq.PUSH)
        self.sock.setsockopt(zmq.SNDHWM, send_hwm)
        self.sock.setsockopt(zmq.LINGER, lingerms)
        self.sock.setsockopt(zmq.IMMEDIATE, 1)
        self.sock.bind(bind_address)
        self.btid = btid
        self.shm_slots = shm_slots
        self.shm_key = shm_key
        self._ring = None

    def publish(self, **kwargs):
        """Send ``{'btid': btid, **kwargs}`` (values must be picklable)."""
        img = kwargs.get(self.shm_key) if self.shm_slots else None
        if isinstance(img, np.ndarray) and img.dtype == np.uint8:
            if self._ring is None:
                self._ring = shm.ShmRing(f'blendtorch-{os.getpid()}-{self.btid}', self.shm_slots, img.nbytes)
            slot, off, h, w, c, gen = self._ring.put(img)
            kwargs = {k: v for k, v in kwargs.items() if k != self.shm_key}
            kwargs[shm.KEY] = (self._ring.name, slot, off, h, w, c, self.shm_key, gen)
        self.sock.send_pyobj({'btid': self.btid, **kwargs})

    def close(self):
        self.sock.close()
        if self._ring is not None:
            self._ring.close()
            self._ring = None
