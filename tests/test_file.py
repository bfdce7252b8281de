"""`.btr` record/replay (reference: tests/test_file.py:4-12) + byte layout."""
import io
import pickle

import numpy as np
import pytest

from blendtorch.btt.file import FileReader, FileRecorder
from blendtorch import btt


@pytest.mark.background
def test_file_recorder_reader(tmp_path):
    with FileRecorder(outpath=tmp_path / 'record.mpkl', max_messages=10) as rec:
        for i in range(7):
            rec.save({'value': i}, is_pickled=False)
    r = FileReader(tmp_path / 'record.mpkl')
    assert len(r) == 7
    for i in range(7):
        assert r[i]['value'] == i


def test_header_is_numpy1_layout(tmp_path):
    """Header = pickle protocol 3 of int64[capacity] written as numpy 1.x does
    (module path numpy.core.multiarray) -> identical to numpy 2's bytes with
    the module path swapped, and stable in size between open and close."""
    path = tmp_path / 'h.btr'
    with FileRecorder(path, max_messages=5) as rec:
        rec.save(b'\x80\x03K\x07.', is_pickled=True)
        rec.save([1, 2], is_pickled=False)
    raw = path.read_bytes()
    offs = np.full(5, -1, np.int64)
    ref_hdr = pickle.dumps(offs, protocol=3).replace(b'numpy._core.multiarray', b'numpy.core.multiarray')
    hdr_len = len(ref_hdr)
    offs[0], offs[1] = hdr_len, hdr_len + 5
    expect = pickle.dumps(offs, protocol=3).replace(b'numpy._core.multiarray', b'numpy.core.multiarray')
    assert raw[:hdr_len] == expect
    assert raw[hdr_len:hdr_len + 5] == b'\x80\x03K\x07.'
    r = FileReader(path)
    assert len(r) == 2 and r[0] == 7 and r[1] == [1, 2]


def test_capacity_limit_and_header_size_100k(tmp_path):
    path = tmp_path / 'c.btr'
    with FileRecorder(path, max_messages=3) as rec:
        for i in range(10):
            rec.save(i)
    assert len(FileReader(path)) == 3
    hdr = pickle.dumps(np.full(100000, -1, np.int64), protocol=3)
    assert len(hdr) - 1 == 800159     # numpy.core path is one byte shorter


def test_file_dataset_concat_and_transform(tmp_path):
    for w in range(3):
        with FileRecorder(FileRecorder.filename(tmp_path / 'rec', w), max_messages=10) as rec:
            for i in range(4):
                rec.save({'w': w, 'i': i})
    ds = btt.FileDataset(tmp_path / 'rec', item_transform=lambda d: (d['w'], d['i']))
    assert len(ds) == 12
    assert ds[0] == (0, 0) and ds[5] == (1, 1) and ds[11] == (2, 3)
    with pytest.raises(AssertionError):
        btt.FileDataset(tmp_path / 'nope')


def test_reader_in_dataloader_workers(tmp_path):
    import torch.utils.data as tud
    with FileRecorder(FileRecorder.filename(tmp_path / 'r', 0), max_messages=16) as rec:
        for i in range(16):
            rec.save({'x': np.full((2, 2), i, np.float32)})
    ds = btt.FileDataset(tmp_path / 'r')
    dl = tud.DataLoader(ds, batch_size=4, num_workers=2, shuffle=True)
    seen = sorted(int(v) for b in dl for v in b['x'][:, 0, 0])
    assert seen == list(range(16))


class _Numpy1OnlyUnpickler(__import__('pickle').Unpickler):
    """What a numpy 1.x reader can resolve: no ``numpy._core`` module path."""

    def find_class(self, module, name):
        if module.startswith('numpy._core'):
            raise __import__('pickle').UnpicklingError(f'numpy 1.x cannot import {module}.{name}')
        return super().find_class(module, name)


def _load_all_numpy1(path):
    import io
    from blendtorch.btt.file import FileReader
    data = open(path, 'rb').read()
    assert b'numpy._core' not in data
    hdr = _Numpy1OnlyUnpickler(io.BytesIO(data)).load()
    offs = FileReader.read_offsets(path)
    assert list(offs) == list(hdr[:len(offs)])
    return [_Numpy1OnlyUnpickler(io.BytesIO(data[int(o):])).load() for o in offs]


@pytest.mark.background
def test_repickled_messages_are_numpy1_readable(tmp_path, free_port):
    """Recordings of shared-memory producer frames (materialised, then
    re-pickled) and DeviceReplayBuffer.save_recordings contain no numpy 2
    module path: a numpy-1 reader loads every message."""
    import numpy as np
    import torch
    from blendtorch import btt
    from blendtorch.btt.replay import DeviceReplayBuffer
    with btt.BlenderLauncher(producer='cubesim', num_instances=1, named_sockets=['DATA'], start_port=free_port,
                             proto='ipc', seed=3,
                             instance_args=[['--mode', 'rgb', '--resolution', '64x48', '--shm', '6']]) as bl:
        ds = btt.RemoteIterableDataset(bl.launch_info.addresses['DATA'], max_items=6,
                                       record_path_prefix=tmp_path / 'shm')
        live = list(ds)
    msgs = _load_all_numpy1(tmp_path / 'shm_00.btr')
    assert len(msgs) == 6
    for m, it in zip(msgs, live):
        assert np.array_equal(m['image'], it['image']) and m['frameid'] == it['frameid']
        assert m['xy'].dtype == np.float64 and m['xy'].shape == (8, 2)
    rb = DeviceReplayBuffer(4, device='cpu')
    rb.extend(torch.arange(4, dtype=torch.uint8).view(4, 1, 1, 1).expand(4, 3, 5, 4).contiguous(),
              frameid=np.arange(4), xy=np.arange(16, dtype=np.float64).reshape(4, 2, 2))
    [path] = rb.save_recordings(str(tmp_path / 'hbm'))
    msgs = _load_all_numpy1(path)
    assert [int(m['frameid']) for m in msgs] == [0, 1, 2, 3]
    assert all(m['image'].shape == (3, 5, 4) and int(m['image'][0, 0, 0]) == i for i, m in enumerate(msgs))
