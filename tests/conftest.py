import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / 'pytorch-blender_amd'))
sys.path.insert(0, str(ROOT / 'tests'))


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP device) -- run with -m gpu')
    config.addinivalue_line('markers', 'background: compatible with headless (Blender --background) runs')
    config.addinivalue_line('markers', 'slow: long-running integration test')


@pytest.fixture(scope='session', autouse=True)
def _native_build():
    """Build the in-tree native components once per session (incremental)."""
    from blendtorch import _build
    import torch
    _build.build_native()
    if _build.hip_available():
        _build.build_hip()
    yield


_port = [30000 + (os.getpid() * 37) % 20000]


@pytest.fixture
def free_port():
    """A base port unlikely to collide across tests/workers (blocks of 20)."""
    import socket
    while True:
        base = _port[0]
        _port[0] += 20
        if _port[0] > 60000:
            _port[0] = 30000
        ok = True
        for p in range(base, base + 20):
            s = socket.socket()
            try:
                s.bind(('127.0.0.1', p))
            except OSError:
                ok = False
            finally:
                s.close()
            if not ok:
                break
        if ok:
            return base
