"""``.btr`` record/replay files.

Format (byte-compatible with the reference, pkg_pytorch/blendtorch/btt/
file.py:10-132):

    [header]  pickle protocol 3 of an int64[capacity] ndarray of message
              offsets, -1 = unused; written as numpy 1.x does (module path
              ``numpy.core.multiarray``) so files stay readable by the
              reference's numpy 1.x stack and by numpy 2
    [msg 0]   pickled message, stored exactly as received (any protocol)
    [msg 1]   ...

The header is written once at open (all -1) and rewritten in place at close;
the array shape and dtype do not change, so neither does its byte length.
"""
import io
import logging
import pickle
from pathlib import Path

import numpy as np

_logger = logging.getLogger('blendtorch')


def _header_bytes(offsets):
    """Pickled offset header, numpy-1.x byte layout."""
    try:
        from .. import _native
        return _native.btr_header(np.ascontiguousarray(offsets, dtype=np.int64))
    except ImportError:  # pure-Python fallback: patch the module path
        raw = pickle.dumps(np.asarray(offsets, dtype=np.int64), protocol=3)
        return raw.replace(b'cnumpy._core.multiarray\n', b'cnumpy.core.multiarray\n', 1)


class FileRecorder:
    """Record messages (raw pickled bytes or objects) into one ``.btr`` file.

    Use as a context manager; ``save`` appends while capacity lasts.
    """

    def __init__(self, outpath='blendtorch.mpkl', max_messages=100000):
        outpath = Path(outpath)
        outpath.parent.mkdir(parents=True, exist_ok=True)
        self.outpath = outpath
        self.capacity = int(max_messages)
        self.file = None
        _logger.info(f'Recording configured for path {outpath}, max_messages {max_messages}.')

    def save(self, data, is_pickled=False):
        """Append ``data`` (bytes if ``is_pickled`` else any picklable object)."""
        if self.num_messages >= self.capacity:
            return
        self.offsets[self.num_messages] = self.file.tell()
        self.num_messages += 1
        if is_pickled:
            self.file.write(data)
        else:
            # protocol 3: readable by Blender 2.8x's Python 3.7
            self.file.write(pickle.dumps(data, protocol=3))

    def __enter__(self):
        self.file = io.open(self.outpath, 'wb', buffering=0)
        self.offsets = np.full(self.capacity, -1, dtype=np.int64)
        self.num_messages = 0
        self.file.write(_header_bytes(self.offsets))
        return self

    def __exit__(self, *args):
        self.file.seek(0)
        self.file.write(_header_bytes(self.offsets))
        self.file.close()
        self.file = None

    @staticmethod
    def filename(prefix, worker_idx):
        """Per-worker recording file name ``{prefix}_{worker_idx:02d}.btr``."""
        return f'{prefix}_{worker_idx:02d}.btr'


class FileReader:
    """Random access to the messages of a ``.btr`` file.

    The file is opened lazily on first access so a reader can be created in
    the parent and used inside forked DataLoader workers.
    """

    def __init__(self, path):
        self.path = path
        self.offsets = FileReader.read_offsets(path)
        self._file = None

    def __len__(self):
        return len(self.offsets)

    def __getitem__(self, idx):
        if self._file is None:
            self._file = io.open(self.path, 'rb', buffering=0)
            self._unpickler = pickle.Unpickler(self._file)
        self._file.seek(int(self.offsets[idx]))
        return self._unpickler.load()

    def close(self):
        if self._file is not None:
            self._file.close()
            self._file = None

    def __getstate__(self):  # picklable for DataLoader workers (spawn)
        d = dict(self.__dict__)
        d['_file'] = None
        d.pop('_unpickler', None)
        return d

    @staticmethod
    def read_offsets(fname):
        """Offsets of the stored messages (header truncated at the first -1)."""
        assert Path(fname).exists(), f'Cannot open {fname} for reading.'
        with io.open(fname, 'rb') as f:
            offsets = pickle.Unpickler(f).load()
        unused = np.flatnonzero(offsets == -1)
        return offsets[:unused[0]] if len(unused) else offsets
