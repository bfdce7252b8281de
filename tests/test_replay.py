"""DeviceReplayBuffer: .btr recordings / streams -> frame store -> sampled,
decoded batches.  CPU variants run the fp32 reference ops; the GPU variants
check the fused gather+decode kernel against them bit for bit."""
import numpy as np
import pytest
import torch
from torch.utils import data

from blendtorch import btt, ops
from blendtorch.btt.replay import DeviceReplayBuffer


def _record(tmp_path, free_port, n=24):
    prefix = str(tmp_path / 'rec')
    with btt.BlenderLauncher(producer='cubesim', num_instances=2, named_sockets=['DATA'], start_port=free_port,
                             seed=7, instance_args=[['--mode', 'rgba']] * 2) as bl:
        ds = btt.RemoteIterableDataset(bl.launch_info.addresses['DATA'], max_items=n, record_path_prefix=prefix)
        items = [x for x in data.DataLoader(ds, batch_size=None, num_workers=0)]
    assert len(items) == n
    return prefix, items


def test_replay_cpu_from_recordings(tmp_path, free_port):
    prefix, items = _record(tmp_path, free_port)
    rb = DeviceReplayBuffer.from_recordings(prefix, device='cpu', chunk=5)
    assert len(rb) == 24 and rb.frame_shape == (480, 640, 4) and rb.nbytes == 24 * 480 * 640 * 4
    # insertion order = recording order (one file, one worker)
    for i in (0, 7, 23):
        assert np.array_equal(rb.store[i].numpy(), np.asarray(items[i]['image']))
        assert int(rb.meta['frameid'][i]) == items[i]['frameid'] and int(rb.meta['btid'][i]) == items[i]['btid']
    cfg = ops.DecodeConfig.densityopt(channels='rgb', gamma=2.2)
    idx = torch.tensor([3, 3, 11, 0])
    b = rb.gather(idx, cfg)
    ref = ops.reference_decode(torch.from_numpy(np.stack([np.asarray(items[i]['image']) for i in idx.tolist()])), cfg)
    assert torch.equal(b['image'], ref)
    assert b['frameid'].tolist() == [items[i]['frameid'] for i in idx.tolist()]
    seen = torch.cat([bb['index'] for bb in rb.batches(8, cfg, shuffle=True, generator=torch.Generator().manual_seed(0))])
    assert sorted(seen.tolist()) == list(range(24))
    s = rb.sample(5, cfg, generator=torch.Generator().manual_seed(1))
    assert s['image'].shape == (5, 3, 480, 640)


def test_replay_ring_semantics():
    rb = DeviceReplayBuffer(4, device='cpu')
    frames = torch.arange(6, dtype=torch.uint8).view(6, 1, 1, 1).expand(6, 2, 2, 1).contiguous()
    rb.extend(frames[:3], frameid=np.arange(3))
    rb.extend(frames[3:], frameid=np.arange(3, 6))
    assert len(rb) == 4
    # slots hold frames 4, 5, 2, 3 (oldest overwritten)
    assert rb.store[:, 0, 0, 0].tolist() == [4, 5, 2, 3] and rb.meta['frameid'].tolist() == [4, 5, 2, 3]
    with pytest.raises(ValueError):
        rb.extend(torch.zeros((1, 3, 3, 1), dtype=torch.uint8), frameid=np.zeros(1))
    with pytest.raises(ValueError):
        rb.extend(frames[:1])   # metadata keys must match


@pytest.mark.gpu
def test_replay_gpu_gather_decode(tmp_path, free_port):
    dev = torch.device('cuda', 0)
    prefix, items = _record(tmp_path, free_port)
    rb = DeviceReplayBuffer.from_recordings(prefix, device=dev, chunk=8)
    assert rb.store.is_cuda and len(rb) == 24
    host = torch.from_numpy(np.stack([np.asarray(it['image']) for it in items]))
    assert torch.equal(rb.store.cpu(), host)
    for cfg in (ops.DecodeConfig.densityopt(channels='rgb', gamma=2.2),
                ops.DecodeConfig.unit(channels='bgr', dtype='bfloat16', layout='nhwc'),
                ops.DecodeConfig(channels='rgba', gamma=2.2, dtype='uint8')):
        idx = torch.tensor([5, 0, 23, 5, 17, 2, 9, 11], device=dev)
        got = rb.gather(idx, cfg)['image']
        ref = ops.reference_decode(host[idx.cpu()], cfg)
        assert torch.equal(got.cpu().float(), ref.float()), cfg
        assert torch.equal(got, ops.decode(rb.store[idx], cfg))
    n = sum(len(b['index']) for b in rb.batches(8, ops.DecodeConfig.unit(), epochs=2))
    assert n == 48


@pytest.mark.gpu
def test_replay_gpu_fill_from_device_loader(free_port):
    from blendtorch.btt.gpu import DeviceLoader
    dev = torch.device('cuda', 0)
    with btt.BlenderLauncher(producer='cubesim', num_instances=2, named_sockets=['DATA'], start_port=free_port,
                             proto='ipc', instance_args=[['--mode', 'rgba', '--shm', '16']] * 2) as bl:
        dl = DeviceLoader(bl.launch_info.addresses['DATA'], batch_size=8, max_items=32, device=dev,
                          decode=ops.DecodeConfig.raw())
        rb = DeviceReplayBuffer(64, device=dev).fill_from(dl, 32)
    assert len(rb) == 32 and rb.frame_shape == (480, 640, 4)
    assert set(rb.meta) >= {'btid', 'frameid', 'xy'}
    b = rb.sample(16, ops.DecodeConfig.unit(channels='rgb', gamma=2.2))
    assert b['image'].shape == (16, 3, 480, 640) and b['xy'].shape == (16, 8, 2)


@pytest.mark.gpu
def test_replay_graphed_sampler():
    """The HIP-graph-captured sampler returns fresh random batches whose
    images equal the eager decode of the indices it drew."""
    dev = torch.device('cuda', 0)
    rb = DeviceReplayBuffer(64, device=dev)
    g = torch.Generator(device=dev).manual_seed(3)
    rb.extend(torch.randint(0, 256, (64, 48, 64, 4), dtype=torch.uint8, device=dev, generator=g),
              frameid=torch.arange(64, device=dev))
    cfg = ops.DecodeConfig.unit(channels='rgb', gamma=2.2)
    sample = rb.graphed_sampler(8, cfg)
    seen = []
    for _ in range(5):
        b = sample()
        idx = b['index'].clone()
        seen.append(idx)
        assert torch.equal(b['image'], ops.decode(rb.store[idx], cfg))
        assert torch.equal(b['frameid'], idx)
    assert len({tuple(i.tolist()) for i in seen}) > 1   # new indices every replay


def test_replay_save_recordings_roundtrip(tmp_path):
    """Frames in a (ring-wrapped) buffer -> .btr files -> FileDataset and
    from_recordings give back the same frames and metadata, oldest first."""
    rb = DeviceReplayBuffer(5, device='cpu')
    frames = torch.arange(7, dtype=torch.uint8).view(7, 1, 1, 1).expand(7, 4, 6, 3).contiguous()
    rb.extend(frames, frameid=np.arange(7), xy=np.arange(7 * 4, dtype=np.float64).reshape(7, 2, 2))
    paths = rb.save_recordings(str(tmp_path / 'hbm'), files=2)
    assert len(paths) == 2
    ds = btt.FileDataset(str(tmp_path / 'hbm'))
    got = sorted((int(it['frameid']), int(it['image'][0, 0, 0]), it['xy'].tolist()) for it in ds)
    assert [g[0] for g in got] == [2, 3, 4, 5, 6]            # the 5 newest survive the ring
    assert all(g[0] == g[1] for g in got)
    assert got[0][2] == np.arange(8, 12, dtype=np.float64).reshape(2, 2).tolist()
    back = DeviceReplayBuffer.from_recordings(str(tmp_path / 'hbm'), device='cpu', meta_keys=('frameid',))
    assert len(back) == 5 and sorted(back.meta['frameid'].tolist()) == [2, 3, 4, 5, 6]


def test_philox_reference_properties():
    """The numpy Philox reference: deterministic, counter-sensitive, in range."""
    a = ops.philox_indices(7, 0, 64, 1000)
    assert a.dtype == np.int64 and a.min() >= 0 and a.max() < 1000
    assert np.array_equal(a, ops.philox_indices(7, 0, 64, 1000))
    assert not np.array_equal(a, ops.philox_indices(7, 64, 64, 1000))
    assert not np.array_equal(a, ops.philox_indices(8, 0, 64, 1000))
    # roughly uniform
    big = ops.philox_indices(1, 0, 40000, 10)
    assert np.bincount(big, minlength=10).min() > 3600


@pytest.mark.gpu
@pytest.mark.parametrize('shape', [(48, 64, 4), (46, 62, 3)])      # vector path / scalar path
def test_replay_fused_sample_kernel(shape):
    """ops.replay_sample: ONE launch draws the Philox indices (== the numpy
    reference), decodes those frames bit-exactly and gathers every metadata
    column (8-byte, 4-byte-multiple and 1-byte rows); the device counter
    advances by B per launch."""
    dev = torch.device('cuda', 0)
    N = 50
    g = torch.Generator(device=dev).manual_seed(0)
    store = torch.randint(0, 256, (N,) + shape, dtype=torch.uint8, device=dev, generator=g)
    meta = {'frameid': torch.arange(N, device=dev) * 3, 'xy': torch.rand(N, 8, 2, device=dev, dtype=torch.float64),
            'flag': torch.arange(N, device=dev) % 3 == 0}
    counter = torch.zeros(2, dtype=torch.int64, device=dev)
    cfgs = [ops.DecodeConfig.densityopt(channels='rgb', gamma=2.2),
            ops.DecodeConfig.unit(channels='bgr', dtype='bfloat16', layout='nhwc'),
            ops.DecodeConfig(channels='rgb', gamma=2.2, dtype='uint8', flip=True)]
    for step, cfg in enumerate(cfgs):
        B = 13
        img, idx, mo = ops.replay_sample(store, N - 3, B, cfg, seed=1234, counter=counter, meta=meta)
        torch.cuda.synchronize()
        expect = ops.philox_indices(1234, step * B, B, N - 3)
        assert idx.cpu().numpy().tolist() == expect.tolist()
        assert counter[0].item() == (step + 1) * B
        ref = ops.reference_decode(store.cpu()[torch.from_numpy(expect)], cfg)
        assert torch.equal(img.cpu(), ref), cfg
        for k, col in meta.items():
            assert torch.equal(mo[k], col[idx]), k
    # a host-side counter value: one launch, nothing advanced on the device
    img, idx, _ = ops.replay_sample(store, N, 7, cfgs[0], seed=5, counter=123)
    assert idx.cpu().tolist() == ops.philox_indices(5, 123, 7, N).tolist() and counter[0].item() == 3 * 13
    # given indices (gather mode) leave the counter alone
    want = torch.tensor([0, N - 1, 7, 7], device=dev)
    img, idx, mo = ops.replay_sample(store, N, 4, cfgs[0], index=want, meta=meta)
    assert torch.equal(idx, want) and counter[0].item() == 3 * 13
    assert torch.equal(img, ops.decode(store[want].contiguous(), cfgs[0]))


@pytest.mark.gpu
def test_replay_buffer_uses_fused_sampler():
    dev = torch.device('cuda', 0)
    rb = DeviceReplayBuffer(32, device=dev, seed=99)
    g = torch.Generator(device=dev).manual_seed(1)
    rb.extend(torch.randint(0, 256, (20, 48, 64, 4), dtype=torch.uint8, device=dev, generator=g),
              frameid=torch.arange(20, device=dev), xy=torch.rand(20, 8, 2, device=dev))
    cfg = ops.DecodeConfig.unit(channels='rgb', gamma=2.2)
    b1, b2 = rb.sample(8, cfg), rb.sample(8, cfg)
    torch.cuda.synchronize()
    assert b1['index'].tolist() == ops.philox_indices(99, 0, 8, 20).tolist()
    assert b2['index'].tolist() == ops.philox_indices(99, 8, 8, 20).tolist()
    for b in (b1, b2):
        assert torch.equal(b['image'], ops.decode(rb.store[b['index']], cfg))
        assert torch.equal(b['frameid'], b['index']) and torch.equal(b['xy'], rb.meta['xy'][b['index']])


def test_table_only_flags_channel_uniform_tables():
    """table_only: 2 (the replay kernel's 32-copy conflict-free table form)
    exactly when the table is in table mode and every output channel has the
    same 256 values; 1 for per-channel tables; 0 for the arithmetic form."""
    import numpy as np
    for cfg in (ops.DecodeConfig.unit(channels='rgb', gamma=2.2),
                ops.DecodeConfig.unit(channels='bgr', dtype='bfloat16', layout='nhwc'),
                ops.DecodeConfig.densityopt(channels='rgb', gamma=2.2),
                ops.DecodeConfig(channels='rgb', mean=[0.1, 0.2, 0.3], std=[1.0, 2.0, 3.0]),
                ops.DecodeConfig(channels='rgba')):
        tab = ops.build_table(cfg)
        if int(tab[ops.XF_HEADER]) != 0:
            want = 0
        else:
            same = all(np.array_equal(tab[:256], tab[256 * c:256 * (c + 1)]) for c in range(1, cfg.cout))
            want = 2 if same else 1
        assert ops.table_only(cfg, torch.device('cpu')) == want, cfg
    assert ops.table_only(ops.DecodeConfig.unit(channels='rgb', gamma=2.2), torch.device('cpu')) == 2
