"""Datasets over live producer streams and over recordings.

Reference: pkg_pytorch/blendtorch/btt/dataset.py:14-153.

* :class:`RemoteIterableDataset` -- ``IterableDataset``; every DataLoader
  worker lazily opens its own PULL socket (RCVHWM = ``queue_size``) connected
  to all producer addresses and yields ``max_items // num_workers`` items.
  Silence longer than ``timeoutms`` fails with
  ``AssertionError('No response within timeout interval.')``.  With a
  ``record_path_prefix`` each worker records raw frames to
  ``{prefix}_{worker:02d}.btr``.
* :class:`SingleFileDataset` / :class:`FileDataset` -- map-style replay of
  one / all recordings matching a prefix (shuffle-capable).

Same-host producers may send images through shared memory (descriptor key
``_btshm``); they are materialised transparently.  A descriptor whose slot
the producer reclaimed while it sat in a queue (lease) is dropped, never
delivered with another frame's pixels.  Frames are decoded with
the native zero-copy unpickler (image arrays are
views over the received buffer); for device-resident batches see
:class:`blendtorch.btt.gpu.DeviceLoader`.
"""
import pickle
from contextlib import ExitStack
from glob import glob

import torch.utils.data as tud

from ..transport import shm, zmq
from .constants import DEFAULT_TIMEOUTMS
from .file import FileReader, FileRecorder


def _identity_item_transform(x):
    return x


class RemoteIterableDataset(tud.IterableDataset):
    """Items streamed from remote producers (``btb.DataPublisher``).

    Params: addresses, queue_size=10, timeoutms=10000, max_items=100000,
    item_transform=None, record_path_prefix=None (as the reference).
    Override :meth:`_item` or pass ``item_transform`` to post-process items.
    """

    def __init__(self, addresses, queue_size=10, timeoutms=DEFAULT_TIMEOUTMS, max_items=100000,
                 item_transform=None, record_path_prefix=None):
        self.addresses = addresses
        self.queue_size = queue_size
        self.timeoutms = timeoutms
        self.max_items = max_items
        self.record_path_prefix = record_path_prefix
        self.item_transform = item_transform or _identity_item_transform

    def enable_recording(self, fname):
        """Record raw frames to ``{fname}_{worker:02d}.btr`` (set before iterating)."""
        self.record_path_prefix = fname

    def stream_length(self, max_items):
        """Set the artificial length of the stream."""
        self.max_items = max_items

    def device_loader(self, batch_size, device=None, decode=None, **kwargs):
        """The MI355X path for this stream: a :class:`blendtorch.btt.gpu.DeviceLoader`
        over the same producers, stream length, timeout and queue size,
        delivering decoded batches in GPU memory instead of host items
        (``item_transform`` and recording do not apply; decode with
        ``decode`` on the GPU, record via ``DeviceReplayBuffer``)."""
        from .gpu import DeviceLoader
        from ..ops import DecodeConfig
        return DeviceLoader(self.addresses, batch_size=batch_size, device=device, max_items=self.max_items,
                            timeoutms=self.timeoutms, rcvhwm=self.queue_size,
                            decode=decode if decode is not None else DecodeConfig(), **kwargs)

    def __iter__(self):
        return self._stream()

    def _stream(self):
        ctx = zmq.Context()
        socket = None
        try:
            socket = ctx.socket(zmq.PULL)
            socket.setsockopt(zmq.RCVHWM, self.queue_size)
            poller = zmq.Poller()
            poller.register(socket, zmq.POLLIN)
            for addr in self.addresses:
                socket.connect(addr)

            wi = tud.get_worker_info()
            worker_id, num_workers = (wi.id, wi.num_workers) if wi is not None else (0, 1)

            with ExitStack() as es:
                rec = None
                if self.record_path_prefix is not None:
                    rec = es.enter_context(FileRecorder(
                        FileRecorder.filename(self.record_path_prefix, worker_id), self.max_items))
                n = 0
                while n < self.max_items // num_workers:
                    ready = dict(poller.poll(self.timeoutms))
                    assert socket in ready, 'No response within timeout interval.'
                    if rec is not None:
                        data = socket.recv()
                        obj = pickle.loads(data)
                        if shm.KEY in obj:   # record the materialised frame
                            obj = shm.resolve(obj)
                            if obj is None:  # stale descriptor: slot reclaimed while queued
                                continue
                            rec.save(obj, is_pickled=False)
                        else:
                            rec.save(data, is_pickled=True)
                    else:
                        obj = shm.resolve(socket.recv_pyobj())
                        if obj is None:
                            continue
                    n += 1
                    yield self._item(obj)
                    del obj
        finally:
            if socket is not None:
                # hand back shared-memory slots of frames still queued here
                try:
                    while socket.poll(0):
                        obj = socket.recv_pyobj()
                        if isinstance(obj, dict) and shm.KEY in obj:
                            shm.release(obj[shm.KEY])
                except Exception:
                    pass
                socket.close()

    def _item(self, item):
        """Transform one received item (default: ``item_transform``)."""
        return self.item_transform(item)


class SingleFileDataset(tud.Dataset):
    """Replay of one ``.btr`` recording."""

    def __init__(self, path, item_transform=None):
        self.reader = FileReader(path)
        self.item_transform = item_transform or _identity_item_transform

    def __len__(self):
        return len(self.reader)

    def __getitem__(self, idx):
        return self._item(self.reader[idx])

    def _item(self, item):
        return self.item_transform(item)


class FileDataset(tud.ConcatDataset):
    """Replay of every recording ``{record_path_prefix}_*.btr`` (sorted)."""

    def __init__(self, record_path_prefix, item_transform=None):
        fnames = sorted(glob(f'{record_path_prefix}_*.btr'))
        assert len(fnames) > 0, f'Found no recording files with prefix {record_path_prefix}'
        super().__init__([SingleFileDataset(f) for f in fnames])
        self.item_transform = item_transform or _identity_item_transform

    def __getitem__(self, idx):
        return self._item(super().__getitem__(idx))

    def _item(self, item):
        return self.item_transform(item)
