"""Producer side of the data stream (reference: btb/publisher.py:4-43).

A PUSH socket that *binds* ``bind_address``: SNDHWM = ``send_hwm``,
LINGER = ``lingerms``, IMMEDIATE = 1 -- so ``publish`` blocks (backpressure)
while no consumer is connected or all consumer queues are full, and no
message is ever dropped.  Every message is the dict
``{'btid': btid, **kwargs}``, pickled.
"""
import itertools
import os

import numpy as np

from ..transport import shm, zmq


_SEGMENTS = itertools.count()


def _segment_name(btid, kind='ring'):
    """Unique per process and publisher (consumers cache mappings by name);
    the ``blendtorch-<pid>-`` prefix is what ``shm.cleanup_pid`` removes."""
    return f'blendtorch-{os.getpid()}-{btid}-{kind}{next(_SEGMENTS)}'


class DataPublisher:
    """Publish rendered images and auxiliary data to ``btt`` datasets.

    ``shm_slots > 0`` (same-host consumers only): u8 ndarrays under
    ``shm_key`` travel through an N-slot shared-memory ring and the message
    carries a small descriptor instead of the pixels.  ``None`` (default)
    takes the value from ``BLENDTORCH_SHM_SLOTS`` (set by
    ``btt.BlenderLauncher(shm_slots=N)``), else 0: plain pickled frames as
    in the reference.

    ``shm_codec='tile16'`` (or ``BLENDTORCH_SHM_CODEC=tile16``) sends ring
    frames as key-frame deltas: the first published image (or the one given
    to :meth:`set_key_frame`, e.g. the empty scene) goes once into a key
    segment, and every frame then carries only the 16x16 tiles that differ
    from it -- lossless, and with a static camera most of the frame never
    crosses PCIe again.  Frames whose size is not a multiple of 16 go raw.
    """

    def __init__(self, bind_address, btid=None, send_hwm=10, lingerms=0, shm_slots=None, shm_key='image',
                 shm_codec=None, shm_lease_s=None):
        if shm_slots is None:
            shm_slots = int(os.environ.get('BLENDTORCH_SHM_SLOTS', '0') or 0)
        if shm_codec is None:
            shm_codec = os.environ.get('BLENDTORCH_SHM_CODEC', 'none') or 'none'
        if shm_codec not in ('none', 'tile16'):
            raise ValueError(f'shm_codec must be none or tile16, not {shm_codec!r}')
        self.shm_codec = shm_codec
        if shm_lease_s is None:
            shm_lease_s = float(os.environ.get('BLENDTORCH_SHM_LEASE_S', '30') or 30)
        self.shm_lease_s = shm_lease_s
        self._key = None
        self._key_ring = None
        self._retired_keys = []   # [(key ring, {slot: generation} still referencing it)]
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
            tiled = self.shm_codec == 'tile16' and shm.tile16_supported(img.shape)
            if self._ring is None:
                c = img.shape[2] if img.ndim == 3 else 1
                cap = max(img.nbytes, shm.tile16_max_bytes(img.shape[0], img.shape[1], c)) if tiled else img.nbytes
                self._ring = shm.ShmRing(_segment_name(self.btid), self.shm_slots, cap, lease_s=self.shm_lease_s)
            if tiled and (self._key is None or self._key.shape != img.shape):
                self.set_key_frame(img)
            if tiled and self._key.shape == img.shape:
                slot, off, h, w, c, gen, _ = self._ring.put_tile16(img, self._key)
                extra = (('tile16', self._key_ring.name, self._key_gen),)
            else:
                slot, off, h, w, c, gen = self._ring.put(img)
                extra = ()
            kwargs = {k: v for k, v in kwargs.items() if k != self.shm_key}
            kwargs[shm.KEY] = (self._ring.name, slot, off, h, w, c, self.shm_key, gen) + extra
        self.sock.send_pyobj({'btid': self.btid, **kwargs})
        if self._retired_keys:
            self._reap_keys()

    def set_key_frame(self, image):
        """Publish ``image`` (u8 HxW[xC]) as the key frame of the tile16 codec.
        It is written once into its own segment; a consumer reads it once.

        May be called mid-stream: frames already published against the old
        key may still sit in queues, so the old key segment stays alive until
        every ring slot that was in use at the change has been handed back
        (its generation moved on); only then is it unlinked."""
        key = np.ascontiguousarray(image, dtype=np.uint8).copy()
        if self._key_ring is not None:
            # a new key gets a new segment: consumers cache keys by segment name
            inflight = {}
            if self._ring is not None:
                for i in range(self._ring.seg.nslots):
                    w = int(self._ring.seg.states[i])
                    if w & 3 in (shm.PUBLISHED, shm.HELD):
                        inflight[i] = w >> 2
            self._retired_keys.append((self._key_ring, inflight))
            self._reap_keys()
        self._key_ring = shm.ShmRing(_segment_name(self.btid, 'key'), 1, key.nbytes)
        _, _, _, _, _, self._key_gen = self._key_ring.put(key)
        self._key = key

    def _reap_keys(self):
        """Unlink retired key segments no in-flight descriptor can name any more."""
        keep = []
        for ring, inflight in self._retired_keys:
            states = self._ring.seg.states if self._ring is not None else None
            for i in list(inflight):
                w = int(states[i]) if states is not None else 0
                if w & 3 == shm.FREE or (w >> 2) != inflight[i]:
                    del inflight[i]     # handed back (or reused): its descriptor is gone
            if inflight:
                keep.append((ring, inflight))
            else:
                ring.close()
        self._retired_keys = keep

    def close(self):
        self.sock.close()
        for ring, _ in self._retired_keys:
            ring.close()
        self._retired_keys = []
        if self._ring is not None:
            self._ring.close()
            self._ring = None
        if self._key_ring is not None:
            self._key_ring.close()
            self._key_ring = None
