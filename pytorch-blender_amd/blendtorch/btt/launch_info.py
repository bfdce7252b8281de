"""Connection information of launched producer instances.

Reference: pkg_pytorch/blendtorch/btt/launch_info.py:4-63.  Only ``addresses``
and ``commands`` are serialised, so another process or host can connect to
running instances.  File-like objects work too (the reference's file-like
branch referenced an un-imported ``nullcontext``; fixed here).
"""
import json
from contextlib import ExitStack, nullcontext


class LaunchInfo:
    """Addresses (``{socket_name: [address per instance]}``), launch commands
    and, when launched locally, the ``subprocess.Popen`` handles."""

    def __init__(self, addresses, commands, processes=None):
        self.addresses = addresses
        self.commands = commands
        self.processes = processes

    def __repr__(self):
        return f'LaunchInfo(addresses={self.addresses!r}, commands={len(self.commands)} commands)'

    @staticmethod
    def _open(file, mode):
        if hasattr(file, 'write' if 'w' in mode else 'read'):
            return nullcontext(file)
        return open(file, mode)

    @staticmethod
    def save_json(file, launch_info):
        """Write addresses and commands as indented JSON to a path or file object."""
        with ExitStack() as stack:
            fp = stack.enter_context(LaunchInfo._open(file, 'w'))
            json.dump({'addresses': launch_info.addresses, 'commands': launch_info.commands}, fp, indent=4)

    @staticmethod
    def load_json(file):
        """Inverse of :meth:`save_json` (processes are not restored)."""
        with ExitStack() as stack:
            fp = stack.enter_context(LaunchInfo._open(file, 'r'))
            data = json.load(fp)
        return LaunchInfo(data['addresses'], data['commands'])
