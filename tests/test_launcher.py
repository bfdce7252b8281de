"""Launcher contract (reference: tests/test_launcher.py) against the headless
Blender stand-in: ids, seeds, sockets, per-instance remainder, LaunchInfo
hand-off to another process, the blendtorch-launch app."""
import json
import multiprocessing as mp
import os
import time
from pathlib import Path

import pytest

from blendtorch import btt
from helpers import BLENDDIR, HEADLESS_BLENDER


def _launch_args(port):
    return dict(scene='', script=str(BLENDDIR / 'launcher.blend.py'), num_instances=2,
                named_sockets=['DATA', 'GYM'], background=True, instance_args=[['--x', '3'], ['--x', '4']],
                seed=10, start_port=port, blend_path=HEADLESS_BLENDER)


def _validate(items):
    assert len(items) == 2
    first, second = (0, 1) if items[0]['btid'] == 0 else (1, 0)
    a, b = items[first]['btargs'], items[second]['btargs']
    assert a['btid'] == 0 and b['btid'] == 1
    assert a['btseed'] == 10 and b['btseed'] == 11
    for x in (a, b):
        assert x['btsockets']['DATA'].startswith('tcp://')
        assert x['btsockets']['GYM'].startswith('tcp://')
    assert items[first]['remainder'] == ['--x', '3']
    assert items[second]['remainder'] == ['--x', '4']


def test_discover_headless_blender():
    info = btt.discover_blender(HEADLESS_BLENDER)
    assert info is not None and info['major'] == 2 and info['minor'] == 90


def test_address_allocation_socket_major(free_port):
    with btt.BlenderLauncher(**_launch_args(free_port)) as bl:
        a = bl.launch_info.addresses
        assert a['DATA'] == [f'tcp://127.0.0.1:{free_port}', f'tcp://127.0.0.1:{free_port + 1}']
        assert a['GYM'] == [f'tcp://127.0.0.1:{free_port + 2}', f'tcp://127.0.0.1:{free_port + 3}']
        assert '-btseed 10' in bl.launch_info.commands[0] and '-btseed 11' in bl.launch_info.commands[1]


@pytest.mark.background
def test_launcher(free_port):
    with btt.BlenderLauncher(**_launch_args(free_port)) as bl:
        ds = btt.RemoteIterableDataset(bl.launch_info.addresses['DATA'], max_items=2)
        _validate([item for item in ds])


def _launch(q, tmp_path, port):
    with btt.BlenderLauncher(**_launch_args(port)) as bl:
        path = Path(tmp_path / 'addresses.json')
        btt.LaunchInfo.save_json(path, bl.launch_info)
        q.put(str(path))
        bl.wait()


@pytest.mark.background
def test_launcher_connected_remote(tmp_path, free_port):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    p = ctx.Process(target=_launch, args=(q, tmp_path, free_port))
    p.start()
    path = q.get(timeout=120)
    info = btt.LaunchInfo.load_json(path)
    ds = btt.RemoteIterableDataset(info.addresses['DATA'], max_items=2)
    _validate([item for item in ds])
    p.join(timeout=60)
    assert p.exitcode == 0


def _run_app(tmp_path, port, bind_addr):
    from blendtorch.btt.apps import launch
    args = _launch_args(port)
    args['bind_addr'] = bind_addr
    with open(tmp_path / 'launchargs.json', 'w') as fp:
        json.dump(args, fp, indent=4)
    launch.main(['--out-launch-info', str(tmp_path / 'launchinfo.json'), str(tmp_path / 'launchargs.json')])


@pytest.mark.background
@pytest.mark.parametrize('bind_addr', ['127.0.0.1', 'primaryip'])
def test_launcher_app(tmp_path, free_port, bind_addr):
    ctx = mp.get_context('spawn')
    p = ctx.Process(target=_run_app, args=(tmp_path, free_port, bind_addr))
    p.start()
    path = tmp_path / 'launchinfo.json'
    t0 = time.time()
    while not path.exists():
        time.sleep(0.1)
        assert time.time() - t0 < 120
    time.sleep(0.2)
    info = btt.LaunchInfo.load_json(path)
    if bind_addr == 'primaryip':
        assert info.addresses['DATA'][0].startswith(f'tcp://{btt.get_primary_ip()}:')
    ds = btt.RemoteIterableDataset(info.addresses['DATA'], max_items=2)
    _validate([item for item in ds])
    p.join(timeout=60)


def test_launch_info_file_objects(tmp_path):
    import io
    info = btt.LaunchInfo({'DATA': ['tcp://a:1']}, ['cmd'])
    buf = io.StringIO()
    btt.LaunchInfo.save_json(buf, info)
    buf.seek(0)
    back = btt.LaunchInfo.load_json(buf)
    assert back.addresses == info.addresses and back.commands == info.commands


def test_missing_blender_raises(tmp_path):
    with pytest.raises(ValueError):
        btt.BlenderLauncher(script='x.py', blend_path=str(tmp_path), num_instances=1)


def test_native_producer_assert_alive_and_teardown(free_port):
    with btt.BlenderLauncher(producer='cubesim', num_instances=2, named_sockets=['DATA'],
                             start_port=free_port) as bl:
        time.sleep(0.3)
        bl.assert_alive()
        pids = [p.pid for p in bl.launch_info.processes]
    for pid in pids:
        with pytest.raises(ProcessLookupError):
            os.kill(pid, 0)


def test_respawn_dead_instance(free_port):
    with btt.BlenderLauncher(producer='cubesim', num_instances=1, named_sockets=['DATA'], start_port=free_port,
                             respawn=True, instance_args=[['--fault', 'exit', '--fault-after', '2']]) as bl:
        ds = btt.RemoteIterableDataset(bl.launch_info.addresses['DATA'], max_items=6, timeoutms=20000)
        items = list(ds)
        assert len(items) == 6
        assert bl.respawn_count >= 1
