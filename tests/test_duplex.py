"""Duplex channel echo (reference: tests/test_duplex.py)."""
import pytest

from blendtorch import btt
from helpers import BLENDDIR, HEADLESS_BLENDER


@pytest.mark.background
def test_duplex(free_port):
    args = dict(scene='', script=BLENDDIR / 'duplex.blend.py', num_instances=2, named_sockets=['CTRL'],
                background=True, start_port=free_port, blend_path=HEADLESS_BLENDER)
    with btt.BlenderLauncher(**args) as bl:
        addresses = bl.launch_info.addresses['CTRL']
        duplex = [btt.DuplexChannel(addr, lingerms=5000) for addr in addresses]
        mids = [d.send(msg=f'hello {idx}') for idx, d in enumerate(duplex)]
        for idx, d in enumerate(duplex):
            dmsg = d.recv(timeoutms=10000)
            assert dmsg['echo']['msg'] == f'hello {idx}'
            assert dmsg['echo']['btid'] is None
            assert dmsg['echo']['btmid'] == mids[idx]
            assert dmsg['btid'] == idx
            dmsg = d.recv(timeoutms=10000)
            assert dmsg['msg'] == 'end'
            assert dmsg['btid'] == idx


def test_duplex_recv_timeout_returns_none(free_port):
    from blendtorch.transport import zmq
    ctx = zmq.Context()
    s = ctx.socket(zmq.PAIR)
    s.bind(f'tcp://127.0.0.1:{free_port}')
    d = btt.DuplexChannel(f'tcp://127.0.0.1:{free_port}')
    assert d.recv(timeoutms=50) is None
    mid = d.send(x=1)
    msg = s.recv_pyobj()
    assert msg == {'btid': None, 'btmid': mid, 'x': 1} and 0 <= mid < 2 ** 32
    s.close()
    d.close()
