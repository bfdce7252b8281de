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


def _identity(x):
    return x


class _Pull:
    """One PULL socket connected to every producer (per DataLoader worker)."""

    def __init__(self, addresses, rcvhwm, timeoutms):
        self.timeoutms = timeoutms
        self.socket = zmq.Context().socket(zmq.PULL)
        self.socket.setsockopt(zmq.RCVHWM, rcvhwm)
        self.poller = zmq.Poller()
        self.poller.register(self.socket, zmq.POLLIN)
        for a in addresses:
            self.socket.connect(a)

    def wait(self):
        if self.socket not in dict(self.poller.poll(self.timeoutms)):
            raise AssertionError('No response within timeout interval.')

    def close(self):
        # frames still queued here may hold producers' shared-memory slots
        try:
            while self.socket.poll(0):
                msg = self.socket.recv_pyobj()
                if isinstance(msg, dict) and shm.KEY in msg:
                    shm.release(msg[shm.KEY])
        except Exception:
            pass
        self.socket.close()


class RemoteIterableDataset(tud.IterableDataset):
    """Items streamed from remote producers (``btb.DataPublisher``).

    Reference semantics (pkg_pytorch/blendtorch/btt/dataset.py:14-117): each
    DataLoader worker opens its own PULL socket (RCVHWM ``queue_size``)
    connected to ALL ``addresses`` and yields ``max_items // num_workers``
    items; silence longer than ``timeoutms`` raises ``AssertionError``; with
    ``record_path_prefix`` every worker records the raw frames it receives to
    ``{prefix}_{worker:02d}.btr``.  Items pass through :meth:`_item`
    (``item_transform``)."""

    def __init__(self, addresses, queue_size=10, timeoutms=DEFAULT_TIMEOUTMS, max_items=100000,
                 item_transform=None, record_path_prefix=None):
        self.addresses = addresses
        self.queue_size = queue_size
        self.timeoutms = timeoutms
        self.max_items = max_items
        self.item_transform = item_transform or _identity
        self.record_path_prefix = record_path_prefix

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
        info = tud.get_worker_info()
        worker, workers = (0, 1) if info is None else (info.id, info.num_workers)
        quota = self.max_items // workers
        pull = _Pull(self.addresses, self.queue_size, self.timeoutms)
        try:
            with ExitStack() as stack:
                rec = None
                if self.record_path_prefix is not None:
                    rec = stack.enter_context(FileRecorder(FileRecorder.filename(self.record_path_prefix, worker),
                                                           self.max_items))
                delivered = 0
                while delivered < quota:
                    pull.wait()
                    obj = self._receive(pull.socket, rec)
                    if obj is None:      # stale shared-memory descriptor: dropped, not counted
                        continue
                    delivered += 1
                    yield self._item(obj)
        finally:
            pull.close()

    @staticmethod
    def _receive(socket, rec):
        """Next message as an object (shared-memory images materialised);
        recorded raw when possible, materialised when it named a ring slot."""
        if rec is None:
            return shm.resolve(socket.recv_pyobj())
        raw = socket.recv()
        obj = pickle.loads(raw)
        if shm.KEY not in obj:
            rec.save(raw, is_pickled=True)
            return obj
        obj = shm.resolve(obj)
        if obj is not None:
            rec.save(obj, is_pickled=False)
        return obj

    def _item(self, item):
        """Transform one received item (default: ``item_transform``)."""
        return self.item_transform(item)


class SingleFileDataset(tud.Dataset):
    """Map-style replay of one ``.btr`` recording."""

    def __init__(self, path, item_transform=None):
        self.reader = FileReader(path)
        self.item_transform = item_transform or _identity

    def __len__(self):
        return len(self.reader)

    def __getitem__(self, idx):
        return self._item(self.reader[idx])

    def _item(self, item):
        return self.item_transform(item)


class FileDataset(tud.ConcatDataset):
    """Replay of every recording ``{record_path_prefix}_*.btr`` (sorted),
    shuffle-capable; ``item_transform`` applies on top."""

    def __init__(self, record_path_prefix, item_transform=None):
        paths = sorted(glob(f'{record_path_prefix}_*.btr'))
        if not paths:
            raise AssertionError(f'Found no recording files with prefix {record_path_prefix}')
        super().__init__([SingleFileDataset(p) for p in paths])
        self.item_transform = item_transform or _identity

    def __getitem__(self, idx):
        return self._item(super().__getitem__(idx))

    def _item(self, item):
        return self.item_transform(item)
