"""Native stand-in producers: cartpolesim protocol, supershapesim duplex loop,
cubesim scenes / lower-left origin / fault hooks, vectorised envs."""
import numpy as np
import pytest
import torch

from blendtorch import btt
from blendtorch.btt.env import VectorRemoteEnv
from blendtorch.models import CartpolePolicy
from blendtorch.transport import zmq


def test_cartpolesim_protocol(free_port):
    with btt.BlenderLauncher(producer='cartpolesim', num_instances=1, named_sockets=['GYM'], start_port=free_port,
                             seed=3) as bl:
        env = btt.env.RemoteEnv(bl.launch_info.addresses['GYM'][0])
        obs, info = env.reset()
        assert len(obs) == 3 and obs[0] == 0.0 and abs(obs[2]) <= 0.6
        assert info['time'] == 2 and info['prev_action'] is None
        t = info['time']
        obs2, r, done, info = env.step(1.5)
        assert r == 0.0 and info['prev_action'] == 1.5 and info['time'] == t + 1
        # a reset after running restarts the episode: cart back at 0
        for _ in range(5):
            env.step(10.0)
        obs3, info3 = env.reset()
        assert obs3[0] == 0.0 and info3['prev_action'] is None
        # numpy actions (gym Box) are accepted
        obs4, *_ = env.step(np.array([0.5], np.float32))
        env.close()


def test_cartpolesim_balances_with_p_controller(free_port):
    with btt.BlenderLauncher(producer='cartpolesim', num_instances=2, named_sockets=['GYM'], start_port=free_port,
                             seed=1) as bl:
        venv = VectorRemoteEnv(bl.launch_info.addresses['GYM'], device='cpu')
        pol = CartpolePolicy()
        obs, _ = venv.reset()
        steps_alive = 0
        for _ in range(100):
            obs, rew, done, _ = venv.step(pol(obs))
            if done.any():
                break
            steps_alive += 1
        assert steps_alive >= 60
        venv.close()


def test_cartpolesim_render(free_port):
    with btt.env.launch_env(scene='', script='', producer='cartpolesim', render_every=2) as env:
        env.reset()
        env.step(0.0)
        img = env.render(mode='rgb_array')
        assert img is not None and img.shape == (270, 480, 3) and img.dtype == np.uint8


def test_supershapesim_duplex_loop(free_port):
    with btt.BlenderLauncher(producer='supershapesim', num_instances=2, named_sockets=['DATA', 'CTRL'],
                             start_port=free_port) as bl:
        remotes = [btt.DuplexChannel(a) for a in bl.launch_info.addresses['CTRL']]
        params = np.tile(np.array([[0, 1, 1, 3, 3, 3]], np.float32), (8, 2, 1))
        params[:, 0, 0] = np.linspace(2, 9, 8)
        ids = np.arange(8)
        for r, p, i in zip(remotes, np.array_split(params, 2), np.array_split(ids, 2)):
            r.send(shape_params=p, shape_ids=i)
        items = list(btt.RemoteIterableDataset(bl.launch_info.addresses['DATA'], max_items=8))
        assert sorted(it['shape_id'] for it in items) == list(range(8))
        assert all(it['image'].shape == (64, 64, 3) for it in items)
        # different frequencies give different images
        imgs = {it['shape_id']: it['image'] for it in items}
        assert not np.array_equal(imgs[0], imgs[7])


@pytest.mark.parametrize('scene', ['cube', 'falling_cubes'])
def test_cubesim_scenes_and_origin(free_port, scene):
    args = dict(producer='cubesim', num_instances=1, named_sockets=['DATA'], seed=4,
                instance_args=[['--scene', scene, '--mode', 'rgba', '--origin', 'lower-left']])
    with btt.BlenderLauncher(start_port=free_port, **args) as bl:
        ctx = zmq.Context()
        s = ctx.socket(zmq.PULL)
        s.connect(bl.launch_info.addresses['DATA'][0])
        assert s.poll(20000)
        m = s.recv_pyobj()
        s.close()
    assert m['image'].shape == (480, 640, 4) and m['origin'] == 'lower-left'
    assert m['xy'].shape == ((8 if scene == 'cube' else 56), 2)
    assert m['image'][..., :3].std() > 3     # something was drawn


def test_cubesim_xy_matches_btb_camera(free_port):
    """cubesim's published vertex projections equal btb.Camera.object_to_pixel
    on the same scene (headless cube preset) for the same cube rotation."""
    from blendtorch.btb import headless
    import blendtorch.btb as btb
    rot = (0.3, 1.1, 2.0)
    bpy = headless.install('cube.blend')
    cube = bpy.data.objects['Cube']
    cube.rotation_euler = rot
    px = btb.Camera().object_to_pixel(cube)
    with btt.BlenderLauncher(producer='cubesim', num_instances=1, named_sockets=['DATA'], start_port=free_port,
                             instance_args=[['--rotation', *map(str, rot)]]) as bl:
        m = next(iter(btt.RemoteIterableDataset(bl.launch_info.addresses['DATA'], max_items=1)))
    np.testing.assert_allclose(m['xy'], px, atol=1e-3)


def test_rigid_world_falls_and_settles():
    """The falling-cubes solver: free fall under gravity, then the cubes come
    to rest on the ground plane (flat on a face: center at plane + half)."""
    from scipy.spatial.transform import Rotation
    from blendtorch import _native
    rng = np.random.default_rng(4)
    n = 7
    c = rng.uniform((-3, -3, 6), (3, 3, 12), size=(n, 3))
    R = Rotation.from_euler('xyz', rng.uniform(-np.pi, np.pi, (n, 3))).as_matrix()
    w = _native.RigidWorld(-2.0)
    w.set_bodies(c, R, np.ones((n, 3)))
    for _ in range(30):
        w.step(1 / 60)
    # free fall for 0.5 s (nothing is near the ground yet): dz = g t^2 / 2 = 1.226
    # (cubes dropped close together may also be nudged apart by contacts)
    drop = c[:, 2] - w.centers()[:, 2]
    assert abs(drop.mean() - 0.5 * 9.81 * 0.25) < 0.05 and drop.min() > 1.0 and drop.max() < 1.45
    for _ in range(600):
        w.step(1 / 60)
    assert w.kinetic_energy() < 0.5
    assert w.min_corner_z() > -2.05
    np.testing.assert_allclose(w.centers()[:, 2], -1.0, atol=0.05)
    Rt = w.rotations()
    np.testing.assert_allclose(Rt @ Rt.transpose(0, 2, 1), np.broadcast_to(np.eye(3), (n, 3, 3)), atol=1e-9)


@pytest.mark.parametrize('producer', ['cubesim', 'blender'])
def test_falling_cubes_fall_within_episode(free_port, producer):
    """falling_cubes: poses are re-dropped at the episode start and then
    evolve under rigid-body physics (projected corners move down the image
    from frame to frame), in the C++ stand-in and in the bpy emulation."""
    from helpers import HEADLESS_BLENDER, ROOT
    ex = ROOT / 'examples' / 'datagen'
    if producer == 'cubesim':
        args = dict(producer='cubesim', instance_args=[['--scene', 'falling_cubes', '--mode', 'rgb']])
    else:
        args = dict(scene=ex / 'falling_cubes.blend', script=ex / 'falling_cubes.blend.py', blend_path=HEADLESS_BLENDER,
                    background=True)
    with btt.BlenderLauncher(num_instances=1, named_sockets=['DATA'], start_port=free_port, seed=3, **args) as bl:
        ctx = zmq.Context()
        s = ctx.socket(zmq.PULL)
        s.connect(bl.launch_info.addresses['DATA'][0])
        msgs = []
        while len(msgs) < 40:
            assert s.poll(30000)
            m = s.recv_pyobj()
            msgs.append(m)
        s.close()
    by_frame = {}
    for m in msgs:
        by_frame.setdefault(int(m['frameid']), m)
    frames = sorted(by_frame)
    assert len(frames) >= 30
    ys = [np.asarray(by_frame[f]['xy'])[:, 1].mean() for f in frames[:30]]
    # falling from z in [6, 12]: the cubes move down the image (pixel y grows)
    assert ys[-1] > ys[0] + 5
    assert all(b >= a - 1e-6 for a, b in zip(ys[:25], ys[1:26]))   # monotone while in free fall


def test_vector_env_step_async_matches_step(free_port):
    """step_async/step_wait (gym VectorEnv style) drive the same deterministic
    trajectories as step(): two identically seeded env sets, one stepped
    synchronously, one asynchronously."""
    trajs = []
    for k, asynchronous in enumerate((False, True)):
        with btt.BlenderLauncher(producer='cartpolesim', num_instances=3, named_sockets=['GYM'],
                                 start_port=free_port + 10 * k, seed=11) as bl:
            venv = VectorRemoteEnv(bl.launch_info.addresses['GYM'])
            obs, _ = venv.reset()
            out = [obs.clone()]
            for t in range(12):
                act = torch.full((3,), 0.5 * ((t % 3) - 1))
                if asynchronous:
                    venv.step_async(act)
                    obs, rew, done, _ = venv.step_wait()
                else:
                    obs, rew, done, _ = venv.step(act)
                out.append(obs.clone())
            venv.close()
        trajs.append(torch.stack(out))
    assert trajs[0].shape == (13, 3, 3)
    torch.testing.assert_close(trajs[0], trajs[1])


def test_vector_env_rgb_batch_cpu(free_port):
    """Rendered frames of all envs come back as one decoded batch (CPU
    reference path here; the GPU test runs the decode kernel)."""
    with btt.BlenderLauncher(producer='cartpolesim', num_instances=2, named_sockets=['GYM'], start_port=free_port,
                             instance_args=[['--render-every', '1']] * 2) as bl:
        venv = VectorRemoteEnv(bl.launch_info.addresses['GYM'])
        venv.reset()
        venv.step(torch.zeros(2))
        rgb = venv.rgb_batch()
        venv.close()
    assert rgb.shape == (2, 3, 270, 480) and rgb.dtype == torch.float32
    assert 0.0 <= float(rgb.min()) and float(rgb.max()) <= 1.0 and float(rgb.std()) > 0


@pytest.mark.parametrize('args', [
    ['--mode', 'rgba'],
    ['--mode', 'rgb', '--origin', 'lower-left'],
    ['--scene', 'falling_cubes', '--mode', 'rgba', '--frame-range', '0', '40'],
    ['--scene', 'falling_cubes', '--mode', 'rgb', '--resolution', '160x120'],
])
def test_cubesim_incremental_render_is_exact(args):
    """Ring-slot frames are rendered incrementally (only the row spans the
    slot's previous frame drew are restored from the cached background): every
    frame must equal a full render byte for byte.  The Cube RGBA stream's
    checksum is pinned: the round-4 render changes (one tone-table load per
    grey pixel, per-row restores) left every byte as before."""
    import json
    import subprocess
    from pathlib import Path
    exe = Path(btt.__file__).resolve().parents[1] / 'bin' / 'cubesim'
    out = subprocess.run([str(exe), '--bench', '120', *args], capture_output=True, text=True, timeout=120)
    rep = json.loads(out.stdout)
    assert out.returncode == 0 and rep['mismatched_bytes'] == 0 and rep['frames'] == 120
    if args == ['--mode', 'rgba']:
        assert rep['checksum'] == 'da5f869cf4aa489d'
