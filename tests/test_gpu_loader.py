"""End-to-end: headless producers -> native receive -> pinned -> HBM -> decode."""
import numpy as np
import pytest
import torch

from blendtorch import btt, ops
from blendtorch.btt.gpu import DeviceLoader
from blendtorch.transport import zmq

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
    assert torch.cuda.is_available()
    ops.hip_ext()
    return torch.device('cuda', 0)


def test_device_loader_cubesim(dev, free_port):
    with btt.BlenderLauncher(producer='cubesim', num_instances=2, named_sockets=['DATA'], start_port=free_port,
                             seed=3, instance_args=[['--mode', 'rgba']] * 2) as bl:
        cfg = ops.DecodeConfig.densityopt(channels='rgb', gamma=2.2)
        dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=8, max_items=64, decode=cfg, device=dev)
        n = 0
        btids = set()
        for b in dl:
            img = b['image']
            assert img.shape == (8, 3, 480, 640) and img.dtype == torch.float32 and img.device == dev
            assert b['btid'].shape == (8,) and b['frameid'].dtype == torch.int64
            assert b['xy'].shape == (8, 8, 2)
            assert float(img.min()) >= -1.0 and float(img.max()) <= 1.0
            btids.update(b['btid'].tolist())
            n += 1
        assert n == 8
        assert btids == {0, 1}
        assert dl.stats['frames'] == 64 and dl.stats['bad'] == 0


def test_device_loader_matches_cpu_decode(dev, free_port):
    """Same frames through the CPU path (pyobj recv + reference decode) and the
    GPU loader must agree bit-exactly: run one producer with a fixed seed
    twice."""
    cfg = ops.DecodeConfig.unit(channels='rgb', gamma=2.2)
    args = dict(producer='cubesim', num_instances=1, named_sockets=['DATA'], seed=11,
                instance_args=[['--mode', 'rgba', '--origin', 'lower-left']])
    with btt.BlenderLauncher(start_port=free_port, **args) as bl:
        ctx = zmq.Context()
        s = ctx.socket(zmq.PULL)
        s.connect(bl.launch_info.addresses['DATA'][0])
        cpu = []
        for _ in range(4):
            assert s.poll(20000)
            cpu.append(s.recv_pyobj())
        s.close()
    with btt.BlenderLauncher(start_port=free_port + 5, **args) as bl:
        dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=4, max_items=4, decode=cfg, device=dev)
        gpu = next(iter(dl))
    imgs = torch.from_numpy(np.stack([np.ascontiguousarray(m['image']) for m in cpu]))
    ref = ops.reference_decode(imgs, cfg, flip=[1, 1, 1, 1])
    assert torch.equal(gpu['image'].cpu(), ref)
    assert gpu['frameid'].tolist() == [m['frameid'] for m in cpu]


def test_device_loader_bad_message_raises(dev, free_port):
    with btt.BlenderLauncher(producer='cubesim', num_instances=1, named_sockets=['DATA'], start_port=free_port,
                             instance_args=[['--fault', 'garbage', '--fault-after', '3']]) as bl:
        dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=2, max_items=8, device=dev)
        with pytest.raises(RuntimeError, match='bad message'):
            for _ in dl:
                pass
