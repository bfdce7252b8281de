"""Observability / configuration helpers."""
import inspect
import os

import torch

import pytest

from blendtorch.btt.gpu import DeviceLoader
from blendtorch.utils import Meter, StreamConfig


def test_stream_config_maps_onto_device_loader():
    """Every StreamConfig field is a DeviceLoader argument with the same
    default, so from_config() and the keyword form build the same loader."""
    params = inspect.signature(DeviceLoader.__init__).parameters
    cfg = StreamConfig()
    for name, value in cfg.kwargs().items():
        assert name in params, name
        assert params[name].default == value, name
    with pytest.raises(ValueError):
        StreamConfig(h2d='dma')
    with pytest.raises(ValueError):
        StreamConfig(batch_size=0)


def test_device_loader_from_config_without_gpu():
    cfg = StreamConfig(batch_size=4, rcvhwm=3, launch_depth=0, log_every=5.0)
    dl = DeviceLoader.from_config(['ipc:///tmp/none'], cfg, device='cuda:0', max_items=40)
    assert (dl.batch_size, dl.rcvhwm, dl.launch_depth, dl.log_every, len(dl)) == (4, 3, 0, 5.0, 10)
    assert dl.io_threads == 1 and dl.metrics() == {}


def test_meter_rates():
    m = Meter()
    m.count('frames', 10)
    with m.time('recv'):
        pass
    d = m.summary()
    assert d['frames'] == 10 and d['frames_per_s'] > 0 and d['recv_ms_avg'] >= 0


def test_trace_range_is_a_shared_no_op_unless_enabled(monkeypatch):
    """The per-batch loops call trace_range: without BLENDTORCH_ROCTX=1 (or
    without a GPU) it must hand back one shared no-op context, not build a
    generator and push roctx ranges (~6 us per call)."""
    import blendtorch.utils as u
    monkeypatch.delenv('BLENDTORCH_ROCTX', raising=False)
    monkeypatch.setattr(u, '_roctx_on', None)
    a, b = u.trace_range('x'), u.trace_range('y')
    assert a is b
    with a:
        pass
    monkeypatch.setenv('BLENDTORCH_ROCTX', '1')
    monkeypatch.setattr(u, '_roctx_on', None)
    assert (u.trace_range('x') is a) == (not torch.cuda.is_available())


def test_bench_thread_report_names_the_python_thread():
    import importlib.util
    from pathlib import Path
    spec = importlib.util.spec_from_file_location('bench_mod', Path(__file__).resolve().parents[1] / 'bench.py')
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    th = bench.thread_cpu()
    assert th[os.getpid()][0] == 'main' and all(isinstance(v[1], int) for v in th.values())


def test_ensure_hw_queues_raises_but_never_lowers(monkeypatch):
    from blendtorch.utils import ensure_hw_queues
    monkeypatch.delenv('BT_HW_QUEUES', raising=False)
    monkeypatch.setenv('GPU_MAX_HW_QUEUES', '4')
    assert ensure_hw_queues(8) == 8 and os.environ['GPU_MAX_HW_QUEUES'] == '8'
    monkeypatch.setenv('GPU_MAX_HW_QUEUES', '16')
    assert ensure_hw_queues(8) == 16
    monkeypatch.setenv('BT_HW_QUEUES', '4')          # an explicit pin wins
    assert ensure_hw_queues(8) == 4 and os.environ['GPU_MAX_HW_QUEUES'] == '4'
    monkeypatch.delenv('BT_HW_QUEUES')
    monkeypatch.delenv('GPU_MAX_HW_QUEUES')
    assert ensure_hw_queues(4) == 4 and 'GPU_MAX_HW_QUEUES' not in os.environ   # HIP's default already


def test_ensure_hw_queues_exact_and_pin_range(monkeypatch):
    """exact=True (graphed training steps) overrides an inherited larger count;
    BT_HW_QUEUES outside 1..32 is refused (the runtime would reject it)."""
    import pytest
    from blendtorch.utils import ensure_hw_queues
    monkeypatch.delenv('BT_HW_QUEUES', raising=False)
    monkeypatch.setenv('GPU_MAX_HW_QUEUES', '8')
    assert ensure_hw_queues(4, exact=True) == 4 and os.environ['GPU_MAX_HW_QUEUES'] == '4'
    monkeypatch.delenv('GPU_MAX_HW_QUEUES')
    assert ensure_hw_queues(4, exact=True) == 4
    for bad in ('0', '33', 'x'):
        monkeypatch.setenv('BT_HW_QUEUES', bad)
        with pytest.raises(ValueError):
            ensure_hw_queues(4)


def test_save_image_matches_torchvision_grid_rules(tmp_path):
    """PNG grids as torchvision.utils.save_image(normalize=True) writes them
    (the densityopt example's image output): min-max over the batch, tiles in
    rows of nrow with 2-pixel zero padding, x * 255 + 0.5 truncated."""
    import numpy as np
    from blendtorch.utils.images import read_png, save_image
    x = torch.arange(3 * 3 * 2 * 2, dtype=torch.float32).reshape(3, 3, 2, 2) - 5
    u8 = save_image(x, tmp_path / 'g.png', nrow=2, normalize=True)
    back = read_png(tmp_path / 'g.png')
    assert back.shape == (2 * 4 + 2, 2 * 4 + 2, 3) and np.array_equal(back, u8)
    lo, hi = float(x.min()), float(x.max())
    want = np.clip((x[1].numpy() - lo) / (hi - lo) * 255 + 0.5, 0, 255).astype(np.uint8).transpose(1, 2, 0)
    assert np.array_equal(back[2:4, 6:8], want)         # tile 1: row 0, column 1
    assert back[:2].max() == 0 and back[8:, 6:].max() == 0   # padding and the empty 4th tile stay 0


def test_loader_window_fairness_and_backlog_fields():
    """DeviceLoader.window: per-producer counts in the timed window, their
    max/min share (bench.py's producer_share_max_over_min) and whether the
    ring's backlog at t0 alone could have served the window."""
    from blendtorch.btt.gpu import DeviceLoader
    s0 = {'t': 0.0, 'frames': 100, 'batches': 10, 'launches': 5, 'image_bytes': 0, 'timed_images': 0,
          'timed_gpu_ms': 0.0, 'consumer_wait_s': 0.0, 'frames_per_btid': {0: 50, 1: 50, 2: 0},
          'ring_slots': 96, 'ring_published': 40, 'ring_held': 8}
    s1 = dict(s0, t=1.0, frames=400, batches=40, frames_per_btid={0: 150, 1: 160, 2: 90},
              ring_published=30)
    w = DeviceLoader.window(s0, s1)
    assert w['producer_frames'] == {0: 100, 1: 110, 2: 90}
    assert w['producer_share_max_over_min'] == round(110 / 90, 4)
    assert w['producers_starved'] == 0
    assert w['backlog_covers_window'] is False            # 40 published < 300 frames
    s1b = dict(s1, frames=130, frames_per_btid={0: 80, 1: 80, 2: 0})
    w = DeviceLoader.window(s0, s1b)
    assert w['producer_share_max_over_min'] is None and w['producers_starved'] == 1
    assert w['backlog_covers_window'] is True             # 40 published >= 30 frames
