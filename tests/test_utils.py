"""Observability / configuration helpers."""
import inspect

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
