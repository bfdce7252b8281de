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
        dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=8, max_items=512, decode=cfg, device=dev)
        # as the reference harness does (benchmarks/benchmark.py:31): let both
        # producers come up -- 512 frames take ~15 ms, less than a process start
        import time
        time.sleep(1.0)
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
        assert n == 64
        # fair-queued fan-in: both producers contribute (the second may start late)
        assert btids == {0, 1}
        assert dl.stats['frames'] == 512 and dl.stats['bad'] == 0


@pytest.mark.parametrize('nprod', [5, 8])
def test_device_loader_fair_across_producers(dev, free_port, nprod):
    """Fair fan-in (reference: examples/datagen/Readme.md:168-177, every
    consumer interleaves all connected producers fairly).  5 producers on the
    loader's 4 IO sockets is the uneven case ({p0,p4},{p1},{p2},{p3}); with
    every producer backpressured (a consumer slower than 5 producers' render
    rate, shm rings full) each producer's share of >= 2000 frames must be
    within +-10 % of 1/P (round 4 drained 64 per socket: 2.04:1)."""
    import time
    args = ['--mode', 'rgba', '--sndhwm', '10', '--shm', '16']
    with btt.BlenderLauncher(producer='cubesim', num_instances=nprod, named_sockets=['DATA'], start_port=free_port,
                             proto='ipc', seed=5, instance_args=[args] * nprod) as bl:
        dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=8, device=dev,
                          decode=ops.DecodeConfig.unit(channels='rgb', gamma=2.2))
        it = iter(dl)
        seen, t0 = set(), time.time()
        while len(seen) < nprod and time.time() - t0 < 60:   # every producer up
            seen.update(next(it)['btid'].tolist())
        assert len(seen) == nprod, seen
        time.sleep(0.5)                                       # rings fill: all backpressured
        s0 = dl.snapshot()
        for _ in range(300):                                  # 2400 frames
            next(it)
            time.sleep(0.0004)                                # <= 20k frames/s: producers stay ahead
        s1 = dl.snapshot()
        it.close()
    w = DeviceLoader.window(s0, s1)
    cnt = w['producer_frames']
    total = sum(cnt.values())
    assert total >= 2000 and sorted(cnt) == list(range(nprod)), cnt
    assert all(abs(c / total - 1 / nprod) <= 0.1 / nprod for c in cnt.values()), cnt
    assert w['producer_share_max_over_min'] is not None and w['producer_share_max_over_min'] <= 1.25, w


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


def test_device_loader_supershape_duplex(dev, free_port):
    """densityopt path: parameters out over the duplex, 64x64 renders back into
    HBM normalised as the reference's item_transform ((x-127.5)/127.5, CHW)."""
    with btt.BlenderLauncher(producer='supershapesim', num_instances=2, named_sockets=['DATA', 'CTRL'],
                             start_port=free_port) as bl:
        remotes = [btt.DuplexChannel(a) for a in bl.launch_info.addresses['CTRL']]
        dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=16, device=dev, max_items=16,
                          decode=ops.DecodeConfig.densityopt(channels='rgb'))
        params = np.tile(np.array([[5, 1, 1, 3, 3, 3]], np.float32), (16, 2, 1))
        for r, p, i in zip(remotes, np.array_split(params, 2), np.array_split(np.arange(16), 2)):
            r.send(shape_params=p, shape_ids=i)
        b = next(iter(dl))
        assert b['image'].shape == (16, 3, 64, 64)
        assert sorted(b['shape_id'].tolist()) == list(range(16))
        assert float(b['image'].min()) >= -1 and float(b['image'].max()) <= 1


def test_vector_env_stages_obs_on_device(dev, free_port):
    from blendtorch.btt.env import VectorRemoteEnv
    from blendtorch.models import CartpolePolicy
    with btt.BlenderLauncher(producer='cartpolesim', num_instances=4, named_sockets=['GYM'],
                             start_port=free_port) as bl:
        venv = VectorRemoteEnv(bl.launch_info.addresses['GYM'], device=dev)
        pol = CartpolePolicy().to(dev)
        obs, _ = venv.reset()
        assert obs.device == dev and obs.shape == (4, 3)
        for _ in range(10):
            obs, rew, done, _ = venv.step(pol(obs))
        assert obs.device == dev
        venv.close()


def test_scatter_loader_single_rank(dev, free_port):
    """Scatter mode on one rank: the root loader lands raw u8 frames, the
    shard is decoded by the gfx950 kernel -- equal to decoding the same
    frames directly -- and the metadata arrives as typed tensors."""
    from blendtorch.parallel import ScatterLoader
    cfg = ops.DecodeConfig.unit(channels='rgb', gamma=2.2)
    with btt.BlenderLauncher(producer='cubesim', num_instances=1, named_sockets=['DATA'], start_port=free_port,
                             instance_args=[['--mode', 'rgba']]) as bl:
        dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=4, max_items=8, device=dev,
                          decode=ops.DecodeConfig.raw(channels='rgb'))
        raw = []

        def tap():
            for b in dl:
                raw.append(b['image'].clone())
                yield b
        sl = ScatterLoader(tap(), 4, cfg, dev, 2)
        out = [b for b in sl]
    assert len(out) == 2 and out[0]['image'].shape == (4, 3, 480, 640) and out[1]['btid'].shape == (4,)
    assert out[0]['xy'].shape == (4, 8, 2) and out[0]['xy'].dtype == torch.float64
    for b, r in zip(out, raw):
        torch.testing.assert_close(b['image'], ops.decode(r, cfg), rtol=0, atol=0)
    assert sl.stats['object_scatters'] == 0


@pytest.mark.parametrize('origin', ['upper-left', 'lower-left'])
def test_device_loader_shared_memory_producer(dev, free_port, origin):
    """Images through the shared-memory ring (descriptor messages) decode to
    exactly what the inline-payload path gives for the same rendered frame."""
    cfg = ops.DecodeConfig.densityopt(channels='rgb', gamma=2.2)
    base = ['--mode', 'rgba', '--rotation', '0.4', '0.9', '1.7', '--origin', origin]
    out, stats = {}, {}
    for i, (k, extra, h2d) in enumerate((('inline', [], 'auto'), ('shm', ['--shm', '12'], 'auto'),
                                         ('shm-copy', ['--shm', '12'], 'copy'))):
        with btt.BlenderLauncher(producer='cubesim', num_instances=2, named_sockets=['DATA'],
                                 start_port=free_port + 5 * i, proto='ipc',
                                 instance_args=[base + extra] * 2) as bl:
            dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=8, max_items=96, decode=cfg, device=dev,
                              h2d=h2d)
            batches = list(dl)
            assert dl.stats['frames'] == 96 and dl.stats['bad'] == 0
            out[k], stats[k] = batches[-1]['image'], dl.stats
            assert 'xy' in batches[0] and batches[0]['xy'].shape == (8, 8, 2)
    torch.testing.assert_close(out['shm'], out['inline'], rtol=0, atol=0)
    torch.testing.assert_close(out['shm-copy'], out['inline'], rtol=0, atol=0)
    # shm frames are registered + mapped: every batch decodes straight from host memory
    assert stats['shm']['direct_batches'] == 12 and stats['shm-copy']['direct_batches'] == 0
    import os
    assert not [f for f in os.listdir('/dev/shm') if f.startswith('blendtorch-')]


def test_device_loader_direct_color4x4(dev, free_port):
    """The MFMA colour-transform kernel on the direct (zero-copy) path equals
    the staged-copy path and the fp32 reference."""
    M = [[0.5, 0.2, 0.1, 0.0], [0.0, 1.0, 0.0, 0.0], [0.1, 0.1, 0.8, 0.0], [0.0, 0.0, 0.0, 1.0]]
    cfg = ops.DecodeConfig(channels='rgba', color_matrix=M, color_bias=(0.1, 0.0, -0.1, 0.0))
    res = {}
    for i, h2d in enumerate(('auto', 'copy')):
        with btt.BlenderLauncher(producer='cubesim', num_instances=1, named_sockets=['DATA'],
                                 start_port=free_port + 5 * i, proto='ipc',
                                 instance_args=[['--mode', 'rgba', '--rotation', '0.1', '0.2', '0.3', '--shm', '8']]) as bl:
            dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=4, max_items=8, decode=cfg, device=dev,
                              h2d=h2d)
            res[h2d] = list(dl)[-1]['image']
            assert dl.stats['direct_batches'] == (2 if h2d == 'auto' else 0)
    torch.testing.assert_close(res['auto'], res['copy'], rtol=0, atol=0)


def _known_frames_producer(addr, n, H=48, W=64, shm_slots=0):
    """A Python producer of n RGBA frames whose pixels are a function of
    their 'k' (so a test can rebuild what the loader decoded)."""
    import threading
    from blendtorch.btb.publisher import DataPublisher

    def frame(k):
        return np.random.default_rng(1000 + k).integers(0, 256, size=(H, W, 4), dtype=np.uint8)

    pub = DataPublisher(addr, btid=1, lingerms=5000, **({'shm_slots': shm_slots} if shm_slots else {}))

    def produce():
        for k in range(n):
            pub.publish(image=frame(k), k=k)

    return threading.Thread(target=produce), pub, frame


@pytest.mark.parametrize('shm', [0, 8])
def test_device_loader_color_jitter_per_image(dev, free_port, shm):
    """Photometric augmentation on the loader path: every image gets its own
    random colour transform inside the MFMA decode (direct path), the batch
    reports the factors, and each image equals the fp32 reference decode with
    those factors (atol 1e-3); the same seed draws the same factors."""
    addr = f'tcp://127.0.0.1:{free_port}'
    jit = ops.ColorJitter(brightness=0.4, contrast=0.4, saturation=0.6, hue=0.2, seed=7)
    cfg = ops.DecodeConfig.unit(channels='rgb', gamma=2.2, color_jitter=jit)
    th, pub, frame = _known_frames_producer(addr, 32, shm_slots=shm)
    dl = DeviceLoader([addr], batch_size=8, max_items=32, device=dev, decode=cfg)
    th.start()
    batches = [dict(image=b['image'].clone(), k=b['k'].clone(), f=b['color_jitter'].clone()) for b in dl]
    th.join()
    pub.close()
    assert len(batches) == 4 and dl.stats['direct_batches'] == 4, dl.stats
    fs = torch.cat([b['f'] for b in batches])
    assert fs.shape == (32, 4) and len({tuple(r.tolist()) for r in fs}) == 32
    assert float(fs[:, :3].min()) >= 0.4 - 1e-6 and float(fs[:, 2].max()) <= 1.6 + 1e-6
    assert float(fs[:, 3].abs().max()) <= 0.2 + 1e-6
    for b in batches:
        x = torch.from_numpy(np.stack([frame(int(k)) for k in b['k']]))
        ref = ops.reference_decode(x, cfg, jitter=b['f'].numpy())
        assert b['image'].shape == (8, 3, 48, 64)
        torch.testing.assert_close(b['image'].cpu(), ref, rtol=1e-4, atol=1e-3)
    # the factors are a function of the seed and the arrival order
    want = ops.jitter_factors(7, [0.4, 0.4, 0.6, 0.2], 32)
    np.testing.assert_allclose(fs.numpy(), want, rtol=0, atol=1e-6)


def test_device_loader_color_matrices_per_position(dev, free_port):
    """DecodeConfig(color_matrices=[B,4,4]): batch position i is decoded
    with transform i, on the direct path."""
    addr = f'tcp://127.0.0.1:{free_port}'
    rng = np.random.default_rng(11)
    M = rng.uniform(-1, 1, size=(4, 4, 4)).astype(np.float32)
    bb = rng.normal(size=(4, 4)).astype(np.float32)
    cfg = ops.DecodeConfig(channels='rgba', gamma=2.2, color_matrices=M, color_biases=bb)
    th, pub, frame = _known_frames_producer(addr, 8)
    dl = DeviceLoader([addr], batch_size=4, max_items=8, device=dev, decode=cfg)
    th.start()
    got = [(b['image'].clone(), b['k'].clone()) for b in dl]
    th.join()
    pub.close()
    assert dl.stats['direct_batches'] == 2
    for img, ks in got:
        x = torch.from_numpy(np.stack([frame(int(k)) for k in ks]))
        ref = ops.reference_color4x4(x, M, bb, gamma=2.2)
        torch.testing.assert_close(img.cpu(), ref, rtol=1e-5, atol=1e-3)


def test_gpu_topology_resolves(dev):
    """hipDeviceGetPCIBusId -> sysfs local_cpulist gives the GPU's NUMA-local CPUs."""
    import os
    from blendtorch.parallel import topology
    bid = topology.gpu_pci_bus_id(0)
    assert bid and len(bid.split(':')) == 3, bid
    plan = topology.plan_rank_cpus(0, 1, sorted(os.sched_getaffinity(0)))
    assert plan['cpus'] and set(plan['cpus']) <= set(os.sched_getaffinity(0))
    print('gpu0', bid, 'numa_local', plan['numa_local'], 'domain size', len(plan['domain']))


@pytest.mark.parametrize('dtype,layout', [('float32', 'nchw'), ('bfloat16', 'nhwc'), ('uint8', 'nchw')])
def test_device_loader_coalesced_launch(dev, free_port, dtype, layout):
    """launch_depth=0 holds direct-path batches until 64 images are pending:
    8 batches of 8 decode in ONE launch through per-image source/destination
    pointers, bit-exact with the one-copy-per-batch path."""
    cfg = (ops.DecodeConfig.unit(channels='rgb', gamma=2.2, dtype=dtype, layout=layout) if dtype != 'uint8'
           else ops.DecodeConfig(channels='rgb', gamma=2.2, dtype=dtype, layout=layout))
    args = ['--mode', 'rgba', '--rotation', '0.3', '0.5', '0.7', '--shm', '48']   # ring > 32 held frames
    res = {}
    for i, (h2d, depth) in enumerate((('auto', 0), ('copy', 2))):
        with btt.BlenderLauncher(producer='cubesim', num_instances=2, named_sockets=['DATA'],
                                 start_port=free_port + 5 * i, proto='ipc', instance_args=[args] * 2) as bl:
            dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=8, max_items=64, decode=cfg, device=dev,
                              h2d=h2d, launch_depth=depth, prefetch=8)
            res[h2d] = [b['image'].clone() for b in dl]
            st = dl.stats
        assert len(res[h2d]) == 8
        if h2d == 'auto':
            assert st['direct_batches'] == 8 and st['launches'] == 1, st
        else:
            assert st['launches'] == 8 and st['direct_batches'] == 0
    for a, b in zip(res['auto'], res['copy']):
        assert torch.equal(a, b)


def _same(a, b):
    if isinstance(b, torch.Tensor):
        return isinstance(a, torch.Tensor) and a.dtype == b.dtype and torch.equal(a, b)
    if isinstance(b, dict):
        return isinstance(a, dict) and a.keys() == b.keys() and all(_same(a[k], b[k]) for k in b)
    if isinstance(b, (list, tuple)):
        return isinstance(a, (list, tuple)) and len(a) == len(b) and all(_same(x, y) for x, y in zip(a, b))
    return a == b


def test_device_loader_native_collate_matches_default_collate(dev, free_port):
    """The loader collates metadata natively; every key must come out exactly
    as torch's default_collate would give it (ints, floats, bools, numpy
    scalars, stacked arrays, strings, nested dicts, ragged arrays)."""
    import threading
    from torch.utils.data import default_collate
    from blendtorch.btb.publisher import DataPublisher
    addr = f'tcp://127.0.0.1:{free_port}'
    pub = DataPublisher(addr, btid=3, lingerms=5000)
    sent = []

    def produce():
        for i in range(8):
            m = dict(image=np.full((16, 32, 4), i, np.uint8), frameid=i, t=0.5 * i, ok=bool(i % 2),
                     f32=np.float32(i) / 3, xy=np.arange(6, dtype=np.float64).reshape(3, 2) + i, name=f'n{i}',
                     info={'a': i, 'b': [i, i + 1]}, ragged=np.zeros(i + 1, np.int16))
            sent.append(m)
            pub.publish(**m)

    th = threading.Thread(target=produce)
    dl = DeviceLoader([addr], batch_size=8, max_items=8, device=dev, decode=ops.DecodeConfig.unit(channels='rgb'))
    th.start()
    b = next(iter(dl))
    th.join()
    pub.close()
    ref = {k: [dict(m, btid=3)[k] for m in sent] for k in list(sent[0]) + ['btid'] if k != 'image'}
    for k, vals in ref.items():
        got = b[k]
        if k == 'ragged':
            assert isinstance(got, list) and all(np.array_equal(g, v) for g, v in zip(got, vals))
            continue
        assert _same(got, default_collate(vals)), k
    assert b['image'].shape == (8, 3, 16, 32)


def test_train_keypoints_example_learns(dev, free_port, tmp_path):
    """examples/datagen/train_keypoints.py: bf16 NHWC frames straight from the
    decode kernel train a CNN on the streamed corner annotations; the loss
    must drop well below its start (the corners are learnable from pixels)."""
    import importlib.util
    import json
    from helpers import ROOT
    spec = importlib.util.spec_from_file_location('train_keypoints', ROOT / 'examples' / 'datagen' / 'train_keypoints.py')
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = tmp_path / 'kp.json'
    mod.main(['--steps', '80', '--batch', '16', '--producers', '4', '--start-port', str(free_port),
              '--json', str(out)])
    res = json.loads(out.read_text())
    assert res['loss_last10'] < 0.5 * res['loss_first10'], res
    assert res['samples_per_s'] if 'samples_per_s' in res else res['value'] > 0


def test_device_loader_survives_producer_crash_with_respawn(dev, free_port):
    """A shared-memory producer that crashes mid-stream (fault injection) is
    respawned by the launcher; the GPU stream keeps going on the survivors
    and the new instance's ring, and no /dev/shm segment is left behind."""
    import os
    # paced producers (300 fps each) so the 800-frame stream outlives the crash and the respawn
    args = [['--mode', 'rgba', '--shm', '16', '--fps', '300'],
            ['--mode', 'rgba', '--shm', '16', '--fps', '300', '--fault', 'exit', '--fault-after', '30']]
    with btt.BlenderLauncher(producer='cubesim', num_instances=2, named_sockets=['DATA'], start_port=free_port,
                             proto='ipc', respawn=True, instance_args=args) as bl:
        dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=8, max_items=800, device=dev,
                          decode=ops.DecodeConfig.unit(channels='rgb'), timeoutms=30000)
        n = sum(1 for _ in dl)
        assert n == 100 and dl.stats['bad'] == 0
        assert bl.respawn_count >= 1
    assert not [f for f in os.listdir('/dev/shm') if f.startswith('blendtorch-')]


@pytest.mark.parametrize('launch_depth', [2, 0])
def test_device_loader_end_to_end_integrity(dev, free_port, launch_depth):
    """Every decoded image belongs to the metadata it is delivered with, and
    no frame is lost or duplicated: 6 stamped producers (3 via the shm ring,
    3 inline over the socket), 6000 frames through direct reads and
    coalesced launches."""
    from collections import defaultdict
    base = ['--mode', 'rgba', '--resolution', '64x48', '--stamp']
    args = [base + (['--shm', '24'] if i % 2 == 0 else []) for i in range(6)]
    with btt.BlenderLauncher(producer='cubesim', num_instances=6, named_sockets=['DATA'], start_port=free_port,
                             proto='ipc', instance_args=args) as bl:
        dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=8, max_items=6000, device=dev,
                          decode=ops.DecodeConfig.raw(), launch_depth=launch_depth, prefetch=8)
        seen = defaultdict(list)
        for b in dl:
            head = b['image'].reshape(8, -1)[:, :16].cpu().numpy()
            for k in range(8):
                st = head[k]
                assert bytes(st[:2]) == b'BT'
                btid = int(st[2]) | (int(st[3]) << 8)
                seq = int(np.frombuffer(st[8:16].tobytes(), '<u8')[0])
                assert btid == int(b['btid'][k]) and seq == int(b['seq'][k]), (btid, seq, b['btid'][k], b['seq'][k])
                seen[btid].append(seq)
        st = dl.stats
    assert sum(len(v) for v in seen.values()) == 6000 and st['bad'] == 0
    for btid, seqs in seen.items():
        assert len(seqs) == len(set(seqs))             # no duplicates
        assert sorted(seqs) == seqs                     # per-producer order preserved
    # fair fan-in puts inline frames into every batch: they land in pinned pool
    # slots (any image-sized frame does), so mixed batches stay on the direct
    # path beside the shm frames read in place from the registered ring
    assert st['shm_frames'] > 0 and st['batches'] == 750
    assert st['direct_batches'] > 0, st


_MATRIX = [
    # (batch, resolution, mode, shm, origin, decode, launch_depth)
    (1, '640x480', 'rgba', True, 'upper-left', 'densityopt', 2),
    (3, '64x48', 'rgb', False, 'upper-left', 'unit', 2),
    (100, '64x48', 'rgba', True, 'upper-left', 'unit', 2),          # > 64 images: staged-copy path
    (8, '62x46', 'rgba', True, 'upper-left', 'unit', 2),            # W % 4 != 0: scalar kernel on host frames
    (8, '64x48', 'rgba', True, 'lower-left', 'densityopt', 0),      # per-image flip in coalesced launches
    (8, '64x48', 'rgba', True, 'upper-left', 'color', 0),           # MFMA colour matrix, coalesced
    (16, '64x48', 'rgba', False, 'lower-left', 'bf16nhwc', 0),      # inline frames, bf16 NHWC, flip
]


@pytest.mark.parametrize('B,res,mode,use_shm,origin,dec,depth', _MATRIX)
def test_device_loader_config_matrix(dev, free_port, B, res, mode, use_shm, origin, dec, depth):
    """Batch sizes, odd widths, inline vs shared-memory frames, flips, dtypes
    and coalescing, all against the fp32 reference decode of the same frame
    (fixed pose: every frame renders identically)."""
    M = [[0.9, 0.1, 0.0, 0.0], [0.0, 1.0, 0.0, 0.0], [0.2, 0.0, 0.8, 0.0], [0.0, 0.0, 0.0, 1.0]]
    cfg = {'densityopt': ops.DecodeConfig.densityopt(channels='rgb', gamma=2.2),
           'unit': ops.DecodeConfig.unit(channels='rgb'),
           'color': ops.DecodeConfig(channels='rgba', gamma=2.2, color_matrix=M, color_bias=(0.0, 0.1, 0.0, 0.0)),
           'bf16nhwc': ops.DecodeConfig.unit(channels='bgr', gamma=2.2, dtype='bfloat16', layout='nhwc')}[dec]
    args = ['--mode', mode, '--resolution', res, '--rotation', '0.3', '0.6', '0.9', '--origin', origin]
    if use_shm:
        args += ['--shm', '128']
    # one reference frame through the CPU path
    with btt.BlenderLauncher(producer='cubesim', num_instances=1, named_sockets=['DATA'], start_port=free_port,
                             proto='ipc', instance_args=[args]) as bl:
        from blendtorch.transport import shm
        s = zmq.Context().socket(zmq.PULL)
        s.connect(bl.launch_info.addresses['DATA'][0])
        assert s.poll(20000)
        frame = np.ascontiguousarray(shm.resolve(s.recv_pyobj())['image'])
        s.close()
    flip = origin == 'lower-left'
    if dec == 'color':
        ref = ops.reference_color4x4(torch.from_numpy(frame[None]), M, cfg.color_bias, gamma=2.2, flip=flip)[0]
        tol = 1e-5   # MFMA accumulation order vs the fp32 reference
    else:
        ref = ops.reference_decode(torch.from_numpy(frame[None]), cfg, flip=[int(flip)])[0]
        tol = 0
    with btt.BlenderLauncher(producer='cubesim', num_instances=2, named_sockets=['DATA'], start_port=free_port + 5,
                             proto='ipc', instance_args=[args] * 2) as bl:
        dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=B, max_items=4 * B, device=dev, decode=cfg,
                          launch_depth=depth, prefetch=4)
        for b in dl:
            img = b['image'].cpu()
            assert img.shape[0] == B
            for k in range(B):
                torch.testing.assert_close(img[k].float(), ref.float(), rtol=0, atol=tol)
        assert dl.stats['bad'] == 0


def test_scene_script_producers_zero_copy(dev, free_port):
    """Unmodified scene scripts (examples/datagen/cube.blend.py under the bpy
    emulation) launched with shm_slots take the zero-copy path into HBM."""
    from helpers import HEADLESS_BLENDER, ROOT
    ex = ROOT / 'examples' / 'datagen'
    with btt.BlenderLauncher(scene=ex / 'cube.blend', script=ex / 'cube.blend.py', num_instances=2,
                             named_sockets=['DATA'], start_port=free_port, background=True,
                             blend_path=HEADLESS_BLENDER, shm_slots=16) as bl:
        dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=4, max_items=32, device=dev,
                          decode=ops.DecodeConfig.unit(channels='rgb', gamma=2.2), timeoutms=60000)
        n = sum(1 for _ in dl)
    assert n == 8 and dl.stats['shm_frames'] == 32 and dl.stats['direct_batches'] == 8


def test_remote_iterable_dataset_device_loader(dev, free_port):
    """RemoteIterableDataset.device_loader: the reference-style dataset object
    hands its stream to the GPU path with the same length/timeout."""
    with btt.BlenderLauncher(producer='cubesim', num_instances=1, named_sockets=['DATA'], start_port=free_port,
                             proto='ipc', shm_slots=16) as bl:
        ds = btt.RemoteIterableDataset(bl.launch_info.addresses['DATA'], max_items=24)
        dl = ds.device_loader(8, device=dev, decode=ops.DecodeConfig.unit(channels='rgb'))
        shapes = [tuple(b['image'].shape) for b in dl]
    assert shapes == [(8, 3, 480, 640)] * 3 and dl.stats['direct_batches'] == 3


def test_vector_env_rgb_batch_gpu(dev, free_port):
    from blendtorch.btt.env import VectorRemoteEnv
    with btt.BlenderLauncher(producer='cartpolesim', num_instances=3, named_sockets=['GYM'], start_port=free_port,
                             instance_args=[['--render-every', '1']] * 3) as bl:
        venv = VectorRemoteEnv(bl.launch_info.addresses['GYM'], device=dev)
        venv.reset()
        venv.step(torch.zeros(3))
        cfg = ops.DecodeConfig.unit(channels='rgb', dtype='bfloat16')
        rgb = venv.rgb_batch(cfg)
        host = np.stack([np.asarray(venv.infos(i)['rgb_array']) for i in range(3)])
        venv.close()
    assert rgb.device == dev and rgb.shape == (3, 3, 270, 480)
    assert torch.equal(rgb.cpu(), ops.reference_decode(torch.from_numpy(host), cfg))


def test_device_loader_metrics(dev, free_port, caplog):
    """metrics(): live while iterating and final afterwards -- per-producer
    provenance, H2D bytes, sampled GPU time per image, coalescing, consumer
    wait; StreamConfig builds the same loader; log_every logs them."""
    import logging
    import time
    from blendtorch.utils import StreamConfig
    with btt.BlenderLauncher(producer='cubesim', num_instances=2, named_sockets=['DATA'], start_port=free_port,
                             seed=5, instance_args=[['--mode', 'rgba']] * 2) as bl:
        cfg = StreamConfig(batch_size=8, log_every=0.0)
        dl = DeviceLoader.from_config(bl.launch_info.addresses['DATA'], cfg, max_items=1024, device=dev,
                                      decode=ops.DecodeConfig.unit(channels='rgb'))
        assert dl.metrics() == {}
        time.sleep(1.0)
        live = None
        with caplog.at_level(logging.INFO, logger='blendtorch'):
            for i, b in enumerate(dl):
                if i == 64:
                    live = dl.metrics()
        m = dl.metrics()
    assert live and 0 < live['frames'] <= m['frames']
    assert m['frames'] == 1024 and m['batches'] == 128 and m['bad'] == 0
    assert set(m['frames_per_producer']) == {0, 1} and sum(m['frames_per_producer'].values()) == 1024
    assert m['h2d_gbytes_per_s'] > 0 and m['frames_per_s'] > 0
    assert m['gpu_us_per_image'] is not None and m['gpu_us_per_image'] > 0
    assert m['images_per_launch'] >= 8 and m['consumer_wait_s'] >= 0
    assert any('DeviceLoader:' in r.getMessage() for r in caplog.records)


@pytest.mark.parametrize('extra,cfg', [
    (['--mode', 'rgba'], dict(channels='rgb', gamma=2.2, scale=1 / 255)),
    (['--mode', 'rgb', '--origin', 'lower-left'], dict(channels='rgb', dtype='bfloat16', layout='nhwc', scale=1 / 255)),
    (['--mode', 'rgba', '--scene', 'falling_cubes'], dict(channels='rgba', dtype='uint8', layout='nhwc')),
])
def test_device_loader_tile_codec(dev, free_port, extra, cfg):
    """Key-frame delta frames (cubesim --codec tile16): the decode kernel
    resolves every 16x16 tile from the HBM key frame or the host payload and
    matches the raw shm path bit for bit, on the direct path and on the copy
    path (host-side rebuild); only the changed tiles cross PCIe."""
    import os
    decode = ops.DecodeConfig(**cfg)
    out, stats = {}, {}
    runs = (('raw', 'none', 'auto'), ('tile', 'tile16', 'auto'), ('tile-copy', 'tile16', 'copy'))
    for i, (k, codec, h2d) in enumerate(runs):
        with btt.BlenderLauncher(producer='cubesim', num_instances=1, named_sockets=['DATA'], seed=7,
                                 start_port=free_port + 5 * i, proto='ipc',
                                 instance_args=[extra + ['--shm', '12', '--codec', codec]]) as bl:
            dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=8, max_items=48, decode=decode,
                              device=dev, h2d=h2d)
            out[k] = torch.cat([b['image'] for b in dl])
            stats[k] = dl.stats
            assert dl.stats['frames'] == 48 and dl.stats['bad'] == 0
    for k in ('tile', 'tile-copy'):
        torch.testing.assert_close(out[k], out['raw'], rtol=0, atol=0)
    assert stats['tile']['tiled_frames'] == 48 and stats['tile']['direct_batches'] == 6
    assert stats['tile-copy']['direct_batches'] == 0
    assert stats['tile']['image_bytes'] < stats['raw']['image_bytes'] / 2
    assert not torch.equal(out['raw'][0], out['raw'][1])   # random poses
    assert not [f for f in os.listdir('/dev/shm') if f.startswith('blendtorch-')]


def test_device_loader_python_publisher_tile16(dev, free_port):
    """A Python producer (btb.DataPublisher, shm_codec='tile16') streams
    key-frame deltas into the GPU loader: decoded batches equal the raw frames
    through the fp32 reference decode, on the fused fill + tile-scatter path."""
    import threading
    from blendtorch.btb.publisher import DataPublisher
    h, w = 48, 64
    bg = (np.arange(h * w * 4, dtype=np.uint32) % 251).astype(np.uint8).reshape(h, w, 4)
    frames = []
    for i in range(16):
        f = bg.copy()
        f[(3 * i) % 38:(3 * i) % 38 + 10, (5 * i) % 52:(5 * i) % 52 + 12] = 200 + i
        frames.append(f)
    addr = f'tcp://127.0.0.1:{free_port}'
    pub = DataPublisher(addr, btid=3, shm_slots=8, shm_codec='tile16')
    pub.set_key_frame(bg)

    def produce():
        for i, f in enumerate(frames):
            pub.publish(image=f, frameid=i)

    t = threading.Thread(target=produce, daemon=True)
    t.start()
    cfg = ops.DecodeConfig.unit(channels='rgb', gamma=2.2)
    got = {}
    try:
        dl = DeviceLoader([addr], batch_size=4, max_items=16, decode=cfg, device=dev, timeoutms=20000)
        for b in dl:
            for img, fid in zip(b['image'], b['frameid'].tolist()):
                got[int(fid)] = img
        t.join(10)
    finally:
        pub.close()
    assert dl.stats['frames'] == 16 and dl.stats['bad'] == 0 and dl.stats['tiled_frames'] == 16
    ref = ops.reference_decode(torch.from_numpy(np.stack(frames)), cfg)
    for i in range(16):
        torch.testing.assert_close(got[i].cpu(), ref[i], rtol=0, atol=0)


def test_device_loader_defer_post_release(dev, free_port):
    """defer_post: buffers are handed back on release() (or at the next
    request when the consumer does not call it); every frame still arrives
    once, in order, with the same pixels as the eager-post loader."""
    args = dict(producer='cubesim', num_instances=1, named_sockets=['DATA'], seed=21,
                instance_args=[['--mode', 'rgba']])
    cfg = ops.DecodeConfig.raw(channels='rgba')
    runs = []
    for defer in (False, True):
        with btt.BlenderLauncher(start_port=free_port + (7 if defer else 0), **args) as bl:
            dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=4, max_items=40, decode=cfg, device=dev,
                              h2d='copy', prefetch=3, defer_post=defer)
            frames, imgs = [], []
            for i, b in enumerate(dl):
                frames += b['frameid'].tolist()
                imgs.append(b['image'].clone())
                if defer and i % 2 == 0:
                    dl.release()
            runs.append((frames, torch.cat(imgs)))
    assert runs[0][0] == runs[1][0] == sorted(runs[1][0]) and len(set(runs[1][0])) == 40
    assert torch.equal(runs[0][1], runs[1][1])


@pytest.mark.parametrize('h2d,decode', [('copy', 'raw'), ('copy', 'unit'), ('auto', 'unit')])
def test_host_sync_many_small_batches_match_cpu(dev, free_port, h2d, decode):
    """host_sync (default): the loader orders itself against the consumer with
    host-side event checks only.  Small frames (which stay cache-resident
    between reuses of a posted buffer) over many batches must still arrive
    exactly as the CPU path receives them."""
    cfg = ops.DecodeConfig.raw(channels='rgba') if decode == 'raw' else ops.DecodeConfig.unit(channels='rgb')
    n = 240
    args = dict(producer='cubesim', num_instances=1, named_sockets=['DATA'], seed=5,
                instance_args=[['--mode', 'rgba', '--resolution', '64x48']])
    port = free_port + {'raw': 0, 'unit': 10}[decode] + (20 if h2d == 'auto' else 0)
    with btt.BlenderLauncher(start_port=port, **args) as bl:
        ctx = zmq.Context()
        s = ctx.socket(zmq.PULL)
        s.connect(bl.launch_info.addresses['DATA'][0])
        cpu = []
        for _ in range(n):
            assert s.poll(20000)
            cpu.append(s.recv_pyobj())
        s.close()
    imgs = torch.from_numpy(np.stack([np.ascontiguousarray(m['image']) for m in cpu]))
    ref = imgs if decode == 'raw' else ops.reference_decode(imgs, cfg)
    with btt.BlenderLauncher(start_port=port + 5, **args) as bl:
        dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=4, max_items=n, decode=cfg, device=dev,
                          h2d=h2d, prefetch=2, host_sync=True)
        got, fids = [], []
        for b in dl:
            got.append(b['image'].float().mean().item())   # consume on the device, as a model would
            fids += b['frameid'].tolist()
            assert torch.equal(b['image'].cpu(), ref[len(fids) - 4:len(fids)]), f'batch ending at {len(fids)}'
    assert fids == [m['frameid'] for m in cpu]


def test_reuse_buffers_ring_rebuilt_per_stream_and_shape(dev, free_port):
    """``reuse_buffers=True``: a second iteration over producers of another
    frame size gets a fresh output ring of the new shape (an old, differently
    sized tensor posted to the native decode would be written out of bounds),
    and within one stream the ring cycles prefetch + 2 tensors."""
    cfg = ops.DecodeConfig.unit(channels='rgb', gamma=2.2)
    dl = DeviceLoader([], batch_size=4, max_items=48, decode=cfg, device=dev, prefetch=2, reuse_buffers=True)
    for k, (w, h) in enumerate(((320, 240), (160, 120))):
        with btt.BlenderLauncher(producer='cubesim', num_instances=1, named_sockets=['DATA'],
                                 start_port=free_port + 5 * k, seed=4,
                                 instance_args=[['--mode', 'rgba', '--resolution', f'{w}x{h}']]) as bl:
            dl.addresses = bl.launch_info.addresses['DATA']
            ptrs = set()
            for b in dl:
                img = b['image']
                assert img.shape == (4, 3, h, w)
                assert float(img.min()) >= 0.0 and float(img.max()) <= 1.0
                ptrs.add(img.data_ptr())
            assert len(ptrs) == dl.prefetch + 2
            assert all(tuple(t.shape) == (4, 3, h, w) for t in dl._ring)
