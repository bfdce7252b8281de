"""``.btr`` record/replay files.

Byte layout (compatible with pkg_pytorch/blendtorch/btt/file.py:10-132)::

    header   pickle protocol 3 of an int64[capacity] ndarray of message
             offsets (-1 = unused), in numpy 1.x's form (module path
             ``numpy.core.multiarray``) so the reference's numpy-1 stack and
             numpy 2 both read it
    body     the messages, each a complete pickle, back to back -- frames
             received from a socket are stored exactly as they arrived

The offset table is written (all -1) when recording starts and rewritten in
place when it ends; shape and dtype never change, so its size does not.

Messages the framework pickles itself (shared-memory frames materialised by
``RemoteIterableDataset``, ``DeviceReplayBuffer.save_recordings``) go through
:func:`dumps_numpy1`: protocol 3 with numpy's globals under their numpy 1.x
module path (``numpy.core.multiarray``), like the reference's own writes
(pkg_pytorch/blendtorch/btt/file.py:46-53 under numpy 1.x).  numpy 2 writes
``numpy._core`` paths that numpy 1 cannot import.
"""
import io
import logging
import pickle
from pathlib import Path

import numpy as np

log = logging.getLogger('blendtorch')


class _Numpy1Pickler(pickle._Pickler):
    """Protocol-3 pickler that names numpy 2's ``numpy._core.*`` globals by
    their numpy 1.x path.  Both numpy generations resolve the result: numpy 2
    still ships ``numpy.core`` as an alias package."""
    _REMAP = {'numpy._core.multiarray': 'numpy.core.multiarray', 'numpy._core.numeric': 'numpy.core.numeric',
              'numpy._core': 'numpy.core'}

    def save_global(self, obj, name=None):
        if name is None:
            name = getattr(obj, '__qualname__', None) or obj.__name__
        module = pickle.whichmodule(obj, name)
        alias = self._REMAP.get(module)
        if alias is None or self.proto >= 4:
            return super().save_global(obj, name)
        self.write(pickle.GLOBAL + f'{alias}\n{name}\n'.encode('utf-8'))
        self.memoize(obj)

    dispatch = dict(pickle._Pickler.dispatch)


def dumps_numpy1(obj):
    """``pickle.dumps(obj, protocol=3)`` readable by numpy 1.x (see module doc)."""
    buf = io.BytesIO()
    _Numpy1Pickler(buf, protocol=3).dump(obj)
    return buf.getvalue()


def _header(offsets):
    """Pickled offset table in numpy 1.x byte layout (native writer when built)."""
    table = np.ascontiguousarray(offsets, dtype=np.int64)
    try:
        from .. import _native
    except ImportError:
        # no native build: CPython's bytes with the module path swapped
        # (same byte count minus the underscore)
        return dumps_numpy1(table)
    return _native.btr_header(table)


class FileRecorder:
    """Append messages to one ``.btr`` file (use as a context manager).

    ``save(data, is_pickled)`` stores raw pickled bytes as they are, or
    pickles ``data`` (protocol 3, numpy 1.x module paths: readable by Blender
    2.8x's Python 3.7 and numpy 1 as well as numpy 2).
    Messages beyond ``max_messages`` are ignored."""

    def __init__(self, outpath='blendtorch.mpkl', max_messages=100000):
        self.outpath = Path(outpath)
        self.outpath.parent.mkdir(parents=True, exist_ok=True)
        self.capacity = int(max_messages)
        self.file = None
        self.offsets = None
        self.num_messages = 0
        log.info('btr recording to %s (capacity %d messages)', self.outpath, self.capacity)

    def __enter__(self):
        self.offsets = np.full(self.capacity, -1, dtype=np.int64)
        self.num_messages = 0
        self.file = open(self.outpath, 'wb', buffering=0)
        self.file.write(_header(self.offsets))
        return self

    def save(self, data, is_pickled=False):
        if self.num_messages == self.capacity:
            return
        payload = data if is_pickled else dumps_numpy1(data)
        self.offsets[self.num_messages] = self.file.tell()
        self.file.write(payload)
        self.num_messages += 1

    def __exit__(self, *exc):
        f, self.file = self.file, None
        f.seek(0)
        f.write(_header(self.offsets))
        f.close()

    @staticmethod
    def filename(prefix, worker_idx):
        """Name of worker ``worker_idx``'s recording: ``{prefix}_{NN}.btr``."""
        return '%s_%02d.btr' % (prefix, worker_idx)


class FileReader:
    """Random access to the messages of a ``.btr`` file.

    The file handle is opened on first access (and dropped when pickled), so
    a reader made in the parent process also works in DataLoader workers."""

    def __init__(self, path):
        self.path = path
        self.offsets = self.read_offsets(path)
        self._fh = None

    def __len__(self):
        return len(self.offsets)

    def __getitem__(self, idx):
        if self._fh is None:
            self._fh = open(self.path, 'rb', buffering=0)
        self._fh.seek(int(self.offsets[idx]))
        return pickle.Unpickler(self._fh).load()

    def close(self):
        fh, self._fh = self._fh, None
        if fh is not None:
            fh.close()

    def __getstate__(self):
        state = dict(self.__dict__)
        state['_fh'] = None
        return state

    @staticmethod
    def read_offsets(fname):
        """Offsets of the stored messages: the header table up to its first -1."""
        if not Path(fname).exists():
            raise AssertionError(f'Cannot open {fname} for reading.')
        with open(fname, 'rb') as f:
            table = pickle.Unpickler(f).load()
        used = int(np.argmax(table == -1)) if (table == -1).any() else len(table)
        return table[:used]
