"""RemoteIterableDataset through DataLoader workers (reference: tests/test_dataset.py)."""
import numpy as np
import pytest
import torch.utils.data as tud

from blendtorch import btt
from helpers import BLENDDIR, HEADLESS_BLENDER, ROOT

BATCH = 4
INSTANCES = 1
WORKERS = 4
NUM_ITEMS = 16


@pytest.mark.background
def test_dataset(free_port):
    args = dict(scene='', script=BLENDDIR / 'dataset.blend.py', num_instances=INSTANCES, named_sockets=['DATA'],
                background=True, start_port=free_port, blend_path=HEADLESS_BLENDER)
    with btt.BlenderLauncher(**args) as bl:
        ds = btt.RemoteIterableDataset(bl.launch_info.addresses['DATA'])
        ds.stream_length(NUM_ITEMS)
        dl = tud.DataLoader(ds, batch_size=BATCH, num_workers=WORKERS, shuffle=False)
        count = 0
        for item in dl:
            assert item['img'].shape == (BATCH, 64, 64)
            assert item['frameid'].shape == (BATCH,)
            count += 1
        assert count == NUM_ITEMS // BATCH


@pytest.mark.background
def test_dataset_recording_and_replay(free_port, tmp_path):
    args = dict(producer='cubesim', num_instances=2, named_sockets=['DATA'], start_port=free_port, seed=5,
                instance_args=[['--mode', 'rgb']] * 2)
    with btt.BlenderLauncher(**args) as bl:
        ds = btt.RemoteIterableDataset(bl.launch_info.addresses['DATA'], max_items=16,
                                       record_path_prefix=tmp_path / 'rec')
        dl = tud.DataLoader(ds, batch_size=4, num_workers=2)
        live = [b for b in dl]
    assert len(live) == 4
    assert sorted(p.name for p in tmp_path.glob('rec_*.btr')) == ['rec_00.btr', 'rec_01.btr']
    replay = btt.FileDataset(tmp_path / 'rec')
    assert len(replay) == 16
    item = replay[3]
    assert item['image'].shape == (480, 640, 3) and item['xy'].shape == (8, 2)
    live_frames = sorted((int(b), int(f)) for batch in live for b, f in zip(batch['btid'], batch['frameid']))
    rep_frames = sorted((replay[i]['btid'], replay[i]['frameid']) for i in range(16))
    assert live_frames == rep_frames


@pytest.mark.background
def test_dataset_timeout_raises(free_port):
    ds = btt.RemoteIterableDataset([f'tcp://127.0.0.1:{free_port}'], max_items=1, timeoutms=300)
    with pytest.raises(AssertionError, match='No response'):
        next(iter(ds))


@pytest.mark.background
def test_item_transform_and_subclass(free_port):
    class MyDS(btt.RemoteIterableDataset):
        def _item(self, item):
            return item['frameid'] * 10

    args = dict(producer='cubesim', num_instances=1, named_sockets=['DATA'], start_port=free_port,
                instance_args=[['--frame-range', '0', '3']])
    with btt.BlenderLauncher(**args) as bl:
        a = list(btt.RemoteIterableDataset(bl.launch_info.addresses['DATA'], max_items=4,
                                           item_transform=lambda d: d['frameid']))
        b = list(MyDS(bl.launch_info.addresses['DATA'], max_items=4))
    assert all(0 <= x <= 3 for x in a)
    assert all(x % 10 == 0 for x in b)


@pytest.mark.background
def test_dataset_shared_memory_producers(free_port):
    """cubesim --shm: descriptors are resolved into images by the CPU dataset;
    slots are handed back (more items than slots flow through)."""
    args = dict(producer='cubesim', num_instances=2, named_sockets=['DATA'], start_port=free_port, proto='ipc',
                instance_args=[['--mode', 'rgb', '--shm', '4', '--rotation', '0.1', '0.2', '0.3']] * 2)
    with btt.BlenderLauncher(**args) as bl:
        # (a generous timeout: the producers start slowly on a loaded host, e.g. under pytest -n)
        ds = btt.RemoteIterableDataset(bl.launch_info.addresses['DATA'], max_items=40, timeoutms=60000)
        items = list(tud.DataLoader(ds, batch_size=4, num_workers=2))
    assert len(items) == 10
    assert items[0]['image'].shape == (4, 480, 640, 3)
    # fixed rotation: every frame identical
    assert (items[0]['image'][0] == items[-1]['image'][-1]).all()


def test_python_publisher_shared_memory(free_port):
    from blendtorch.btb.publisher import DataPublisher
    from blendtorch.transport import shm, zmq
    pub = DataPublisher(f'tcp://127.0.0.1:{free_port}', btid=0, shm_slots=3)
    ctx = zmq.Context()
    pull = ctx.socket(zmq.PULL)
    pull.connect(f'tcp://127.0.0.1:{free_port}')
    for i in range(10):
        img = np.full((8, 6, 3), i, np.uint8)
        pub.publish(image=img, frameid=i)
        msg = pull.recv_pyobj()
        assert shm.KEY in msg and 'image' not in msg
        msg = shm.resolve(msg)
        assert (msg['image'] == i).all() and msg['frameid'] == i
    pub.close()
    pull.close()


def _moving_square_frames(n, h=48, w=64, c=4):
    bg = (np.arange(h * w * c, dtype=np.uint32) % 251).astype(np.uint8).reshape(h, w, c)
    frames = []
    for i in range(n):
        f = bg.copy()
        y, x = (3 * i) % (h - 10), (5 * i) % (w - 12)
        f[y:y + 10, x:x + 12] = 200 + i
        frames.append(f)
    return bg, frames


def test_python_publisher_tile16_codec(free_port):
    """DataPublisher(shm_codec='tile16'): key frame once, then only changed
    16x16 tiles; shm.resolve rebuilds every frame exactly; other sizes go raw."""
    from blendtorch.btb.publisher import DataPublisher
    from blendtorch.transport import shm, zmq
    bg, frames = _moving_square_frames(12)
    pub = DataPublisher(f'tcp://127.0.0.1:{free_port}', btid=0, shm_slots=4, shm_codec='tile16')
    pub.set_key_frame(bg)
    pull = zmq.Context().socket(zmq.PULL)
    pull.connect(f'tcp://127.0.0.1:{free_port}')
    try:
        _check_tile16_stream(pub, pull, frames, free_port)
    finally:
        pub.close()
        pull.close()


def _check_tile16_stream(pub, pull, frames, free_port):
    from blendtorch.btb.publisher import DataPublisher
    from blendtorch.transport import shm
    for i, f in enumerate(frames):
        pub.publish(image=f, frameid=i)
        msg = pull.recv_pyobj()
        desc = msg[shm.KEY]
        assert len(desc) == 9 and desc[8][0] == 'tile16'
        seg = shm._open(desc[0])
        ntiles = int(np.frombuffer(seg.mm, dtype=np.uint32, count=1, offset=desc[2])[0])
        assert 1 <= ntiles <= 4          # a 10x12 square touches at most 2x2 tiles
        msg = shm.resolve(msg)
        assert np.array_equal(msg['image'], f) and msg['frameid'] == i
    pub.publish(image=np.full((10, 6, 3), 7, np.uint8), frameid=99)   # not a multiple of 16: raw
    msg = pull.recv_pyobj()
    assert len(msg[shm.KEY]) == 8
    with pytest.raises(ValueError):
        DataPublisher(f'tcp://127.0.0.1:{free_port + 1}', shm_slots=2, shm_codec='jpeg')


@pytest.mark.parametrize('codec', [None, 'tile16'])
def test_launcher_shm_slots_reaches_scene_scripts(free_port, codec):
    """BlenderLauncher(shm_slots=N[, shm_codec='tile16']) switches an
    unmodified scene script's DataPublisher to the shared-memory ring
    (descriptor messages, key-frame deltas with the codec), and the CPU
    dataset resolves them back into images."""
    from blendtorch.transport import shm, zmq
    ex = ROOT / 'examples' / 'datagen'
    args = dict(scene=ex / 'cube.blend', script=ex / 'cube.blend.py', num_instances=1, named_sockets=['DATA'],
                start_port=free_port, background=True, blend_path=HEADLESS_BLENDER, shm_slots=8, shm_codec=codec)
    with btt.BlenderLauncher(**args) as bl:
        s = zmq.Context().socket(zmq.PULL)
        s.connect(bl.launch_info.addresses['DATA'][0])
        assert s.poll(30000)
        raw = s.recv_pyobj()
        assert shm.KEY in raw and 'image' not in raw
        assert (len(raw[shm.KEY]) == 9 and raw[shm.KEY][8][0] == 'tile16') if codec else len(raw[shm.KEY]) == 8
        shm.release(raw[shm.KEY])
        s.close()
        ds = btt.RemoteIterableDataset(bl.launch_info.addresses['DATA'], max_items=12)
        items = list(ds)
    assert len(items) == 12 and items[0]['image'].shape == (480, 640, 3)


@pytest.mark.background
@pytest.mark.parametrize('extra', [['--mode', 'rgba'], ['--mode', 'rgb', '--origin', 'lower-left', '--stamp'],
                                   ['--mode', 'rgba', '--scene', 'falling_cubes']])
def test_dataset_tile_codec_matches_raw(free_port, extra):
    """cubesim --codec tile16 (key-frame deltas in the shm ring) gives the CPU
    dataset exactly the frames the raw shm path gives for the same seed."""
    from blendtorch.transport import shm
    frames = {}
    pids = []
    for i, codec in enumerate(('none', 'tile16')):
        args = dict(producer='cubesim', num_instances=1, named_sockets=['DATA'], start_port=free_port + 5 * i,
                    proto='ipc', seed=11, instance_args=[extra + ['--shm', '6', '--codec', codec]])
        with btt.BlenderLauncher(**args) as bl:
            pids += [p.pid for p in bl.launch_info.processes]
            ds = btt.RemoteIterableDataset(bl.launch_info.addresses['DATA'], max_items=24)
            frames[codec] = [(it['frameid'], it['image']) for it in ds]
    assert len(frames['tile16']) == 24
    for (fa, a), (fb, b) in zip(frames['none'], frames['tile16']):
        assert fa == fb and a.shape == b.shape and np.array_equal(a, b)
    # frames differ from each other (random poses), so tiles were really sent
    assert not np.array_equal(frames['tile16'][0][1], frames['tile16'][1][1])
    # this test's producers removed their rings (other tests may run concurrently)
    mine = tuple(f'blendtorch-{pid}-' for pid in pids)
    assert not [f for f in __import__('os').listdir('/dev/shm') if f.startswith(mine)]
    del shm
