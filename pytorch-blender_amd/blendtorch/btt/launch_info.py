"""Connection information of launched producer instances.

Reference: pkg_pytorch/blendtorch/btt/launch_info.py:4-63.  Only ``addresses``
and ``commands`` are serialised, so another process or host can connect to
running instances.  File-like objects work too (the reference's file-like
branch referenced an un-imported ``nullcontext``; fixed here).
"""
import json
from contextlib import contextmanager

_SERIALISED = ('addresses', 'commands')


@contextmanager
def _stream(file, mode):
    """Yield ``file`` itself when it is already a file object (left open),
    otherwise the path opened in ``mode`` (closed on exit)."""
    if hasattr(file, 'write' if 'w' in mode else 'read'):
        yield file
        return
    with open(file, mode) as fp:
        yield fp


class LaunchInfo:
    """Addresses (``{socket_name: [address per instance]}``), launch commands
    and, when launched locally, the ``subprocess.Popen`` handles."""

    def __init__(self, addresses, commands, processes=None):
        self.addresses = addresses
        self.commands = commands
        self.processes = processes

    def __repr__(self):
        return f'LaunchInfo(addresses={self.addresses!r}, commands={len(self.commands)} commands)'

    def to_dict(self):
        """The JSON-serialisable part (no process handles)."""
        return {k: getattr(self, k) for k in _SERIALISED}

    @classmethod
    def from_dict(cls, d):
        return cls(*(d[k] for k in _SERIALISED))

    @staticmethod
    def save_json(file, launch_info):
        """Write addresses and commands as indented JSON to a path or file object."""
        with _stream(file, 'w') as fp:
            json.dump(launch_info.to_dict(), fp, indent=4)

    @staticmethod
    def load_json(file):
        """Inverse of :meth:`save_json` (processes are not restored)."""
        with _stream(file, 'r') as fp:
            return LaunchInfo.from_dict(json.load(fp))
