"""GPU loader: slot ownership under consumer pauses, mid-stream key-frame
changes, the multi-stream copy path, timed-window metrics, and proof that
the fused consumer kernels (not the PyTorch fallback) run on the bench
shapes."""
import threading
import time

import numpy as np
import pytest
import torch

from blendtorch import btt, ops
from blendtorch.btt.gpu import DeviceLoader

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    ops.hip_ext()     # fail loudly if the extension is missing on a GPU box
    return torch.device('cuda', 0)


def _check_stamps(b, B):
    head = b['image'].reshape(B, -1)[:, :16].cpu().numpy()
    out = []
    for k in range(B):
        st = head[k]
        assert bytes(st[:2]) == b'BT'
        btid = int(st[2]) | (int(st[3]) << 8)
        seq = int(np.frombuffer(st[8:16].tobytes(), '<u8')[0])
        assert btid == int(b['btid'][k]) and seq == int(b['seq'][k]), (btid, seq, b['btid'][k], b['seq'][k])
        out.append((btid, seq))
    return out


@pytest.mark.parametrize('h2d', ['auto', 'copy'])
def test_consumer_pause_past_lease_never_tears(dev, free_port, h2d):
    """The consumer stops for 8x the producers' lease with slots claimed and
    descriptors queued: no batch ever carries another frame's pixels, the
    stream keeps going, and stale descriptors are only ever dropped."""
    args = [['--mode', 'rgba', '--resolution', '64x48', '--stamp', '--shm', '6', '--lease-ms', '150']] * 2
    with btt.BlenderLauncher(producer='cubesim', num_instances=2, named_sockets=['DATA'], start_port=free_port,
                             proto='ipc', instance_args=args) as bl:
        dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=4, max_items=160, device=dev,
                          decode=ops.DecodeConfig.raw(), h2d=h2d, prefetch=2, timeoutms=30000)
        n = 0
        for i, b in enumerate(dl):
            if i in (3, 20):
                time.sleep(1.2)
                s = dl.snapshot()
                assert s['ring_held'] >= 1          # the loader holds claimed slots through the pause
            _check_stamps(b, 4)
            n += 1
        st = dl.stats
    assert n == 40 and st['shm_torn'] == 0 and st['bad'] == 0


def test_key_frame_change_mid_stream_gpu(dev, free_port):
    """A Python tile16 producer switches key frames twice while frames naming
    the old key are in flight: every decoded image equals the reference
    decode of the raw frame, and replaced keys are freed from HBM."""
    from blendtorch.btb.publisher import DataPublisher
    h, w = 48, 64
    keys = [np.full((h, w, 4), v, np.uint8) for v in (20, 120, 220)]
    frames = []
    for i in range(240):
        f = keys[i // 80].copy()
        f[(3 * i) % 32:(3 * i) % 32 + 16, (5 * i) % 48:(5 * i) % 48 + 16] = (i * 7) % 256
        frames.append(f)
    addr = f'tcp://127.0.0.1:{free_port}'
    pub = DataPublisher(addr, btid=3, shm_slots=12, shm_codec='tile16')

    def produce():
        for i, f in enumerate(frames):
            if i % 80 == 0:
                pub.set_key_frame(keys[i // 80])
            pub.publish(image=f, frameid=i)

    t = threading.Thread(target=produce, daemon=True)
    t.start()
    cfg = ops.DecodeConfig.unit(channels='rgb', gamma=2.2)
    got = {}
    try:
        dl = DeviceLoader([addr], batch_size=1, max_items=240, decode=cfg, device=dev, timeoutms=30000,
                          launch_depth=1)
        for b in dl:
            got[int(b['frameid'][0])] = b['image'][0]
        t.join(10)
        st = dl.stats
    finally:
        pub.close()
    assert sorted(got) == list(range(240))
    ref = ops.reference_decode(torch.from_numpy(np.stack(frames)), cfg)
    for i in range(240):
        torch.testing.assert_close(got[i].cpu(), ref[i], rtol=0, atol=0)
    assert st['tiled_frames'] > 0 and st['bad'] == 0
    assert st['keys_evicted'] >= 1


def test_copy_path_stream_fanout_integrity(dev, free_port):
    """h2d='copy' with the frames of a batch spread over 1, 2 and 4 copy
    streams: every image still matches its metadata, in order per producer."""
    base = ['--mode', 'rgba', '--resolution', '160x96', '--stamp', '--shm', '24']
    for k, cs in enumerate((1, 2, 4)):
        with btt.BlenderLauncher(producer='cubesim', num_instances=3, named_sockets=['DATA'],
                                 start_port=free_port + 5 * k, proto='ipc', instance_args=[base] * 3) as bl:
            dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=8, max_items=1600, device=dev,
                              decode=ops.DecodeConfig.raw(), h2d='copy', copy_streams=cs, prefetch=6)
            seen = {}
            for b in dl:
                for btid, seq in _check_stamps(b, 8):
                    assert seq > seen.get(btid, -1)
                    seen[btid] = seq
            assert dl.stats['direct_batches'] == 0 and dl.stats['frames'] == 1600
            # identity decode on the copy path: DMA straight into the batch tensor, no kernel
            assert dl.stats['passthrough_batches'] == 200


def test_window_metrics_scope(dev, free_port):
    with btt.BlenderLauncher(producer='cubesim', num_instances=2, named_sockets=['DATA'], start_port=free_port,
                             proto='ipc', instance_args=[['--mode', 'rgba', '--shm', '16']] * 2) as bl:
        dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=8, max_items=8 * 400, device=dev,
                          decode=ops.DecodeConfig.unit(channels='rgb'))
        it = iter(dl)
        for _ in range(100):
            next(it)
        torch.cuda.synchronize()
        s0 = dl.snapshot()
        for _ in range(200):
            next(it)
        torch.cuda.synchronize()
        s1 = dl.snapshot()
        it.close()
    w = DeviceLoader.window(s0, s1)
    assert 1590 <= w['frames'] <= 1610 + 8 * 6          # 200 batches (+ what the pipeline ran ahead)
    assert w['frames_per_s'] > 0 and w['h2d_gbytes_per_s'] > 0
    assert w['gpu_us_per_image'] is not None and w['gpu_us_per_image'] > 0
    assert set(w['producer_frames_per_s']) == {0, 1}
    # ring occupancy covers every mapped producer ring (a producer that had not
    # delivered yet at t0 is mapped by t1)
    assert w['ring_t0']['slots'] in (16, 32) and w['ring_t1']['slots'] == 32
    assert 0 <= w['ring_t1']['published'] + w['ring_t1']['held'] <= 32


def test_fused_consumer_kernels_run_on_bench_shapes(dev):
    """bench.py --consumer disc: the discriminator step on 8x{32..256}x240x320
    bf16 NHWC activations must take the gfx950 BN+LeakyReLU and pooling
    kernels -- the modules fall back to PyTorch silently otherwise."""
    from blendtorch.models import Discriminator
    model = Discriminator(nc=3, ndf=32, adaptive=True).to(dev).to(memory_format=torch.channels_last)
    x = torch.rand(8, 480, 640, 3, device=dev).to(torch.bfloat16).permute(0, 3, 1, 2)   # decode output layout
    before = dict(ops.KERNEL_CALLS)
    with torch.autocast('cuda', dtype=torch.bfloat16):
        out = model(x)
    torch.nn.functional.binary_cross_entropy(out.float(), torch.ones_like(out.float())).backward()
    torch.cuda.synchronize()
    d = {k: ops.KERNEL_CALLS.get(k, 0) - before.get(k, 0) for k in ops.KERNEL_CALLS}
    assert d.get('bn_forward') == 4 and d.get('bn_backward') == 4, d
    assert d.get('adaptive_avgpool_nhwc') == 1 and d.get('adaptive_avgpool_nhwc_bwd') == 1, d
    # and each BN layer saw the bench activation shapes in bf16
    shapes = []
    hooks = [m.register_forward_pre_hook(lambda m, a: shapes.append((tuple(a[0].shape), a[0].dtype)))
             for m in model.modules() if isinstance(m, ops.BatchNormLeakyReLU2d)]
    with torch.autocast('cuda', dtype=torch.bfloat16):
        model(x)
    for h in hooks:
        h.remove()
    assert [s for s, _ in shapes] == [(8, 32, 240, 320), (8, 64, 120, 160), (8, 128, 60, 80), (8, 256, 30, 40)]
    assert all(dt == torch.bfloat16 for _, dt in shapes)
    assert all(ops.bn_supported(torch.empty(s, device=dev, dtype=torch.bfloat16)) for s, _ in shapes)


def test_vector_env_staging_survives_busy_stream(dev, free_port):
    """A long kernel is queued before step(): the H2D copies of three steps
    all wait behind it, yet each step's device observations are that step's
    (rotating pinned buffers guarded by events, btt/env.py _PinnedStager)."""
    from blendtorch.btt.env import VectorRemoteEnv
    with btt.BlenderLauncher(producer='cartpolesim', num_instances=3, named_sockets=['GYM'],
                             start_port=free_port) as bl:
        venv = VectorRemoteEnv(bl.launch_info.addresses['GYM'], device=dev)
        venv.reset()
        torch.cuda.synchronize()
        torch.cuda._sleep(200_000_000)          # keeps the stream busy well past the three steps
        outs, hosts = [], []
        for k in range(3):
            obs, _, _, _ = venv.step(torch.full((3,), 0.5 * (k + 1)))
            outs.append(obs)
            hosts.append(np.stack([np.asarray(venv.infos(i)['obs'], np.float32) for i in range(3)]))
        torch.cuda.synchronize()
        venv.close()
    assert not np.array_equal(hosts[0], hosts[1])
    for o, h in zip(outs, hosts):
        assert torch.equal(o.cpu(), torch.from_numpy(h))
