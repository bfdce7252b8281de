"""Remote env protocol (reference: tests/test_env.py).

The reply to request k is the ctx after the frame that applied action k;
``count`` is 1 after reset, done after frame > 10, reset restores obs 0."""
import pytest

from blendtorch import btt
from helpers import BLENDDIR, HEADLESS_BLENDER, ROOT


class MyEnv(btt.env.OpenAIRemoteEnv):
    def __init__(self, background=True, **kwargs):
        super().__init__(version='1.0.0')
        self.launch(scene='', script=BLENDDIR / 'env.blend.py', background=background,
                    blend_path=HEADLESS_BLENDER, **kwargs)


def launch_env_with(monkeypatch, port):
    # route launch_env's BlenderLauncher to the headless blender / a free port
    import blendtorch.btt.env as envmod
    orig = envmod.BlenderLauncher

    def patched(**kw):
        kw.setdefault('start_port', port)
        kw['blend_path'] = HEADLESS_BLENDER
        return orig(**kw)
    monkeypatch.setattr(envmod, 'BlenderLauncher', patched)


def _run_remote_env(background, monkeypatch, port):
    launch_env_with(monkeypatch, port)
    env = btt.env.OpenAIRemoteEnv(version='1.0.0')
    env.launch(scene='', script=BLENDDIR / 'env.blend.py', background=background)
    obs = env.reset()
    assert obs == 0.
    obs, reward, done, info = env.step(0.1)
    assert obs == pytest.approx(0.1)
    assert reward == 0.
    assert not done
    assert info['count'] == 2
    obs, reward, done, info = env.step(0.6)
    assert obs == pytest.approx(0.6)
    assert reward == 1.
    assert not done
    assert info['count'] == 3
    for _ in range(8):
        obs, reward, done, info = env.step(0.6)
    assert done
    obs = env.reset()
    assert obs == 0.
    obs, reward, done, info = env.step(0.1)
    assert obs == pytest.approx(0.1)
    assert reward == 0.
    assert not done
    assert info['count'] == 2
    assert env.env_time is not None
    env.close()


@pytest.mark.background
def test_remote_env(monkeypatch, free_port):
    _run_remote_env(True, monkeypatch, free_port)


def test_remote_env_ui(monkeypatch, free_port):
    _run_remote_env(False, monkeypatch, free_port)


def test_remote_env_render_rgb_array(monkeypatch, free_port):
    launch_env_with(monkeypatch, free_port)
    with btt.env.launch_env(scene='', script=BLENDDIR / 'env.blend.py', background=True, render_every=1) as env:
        obs, info = env.reset()
        env.step(0.3)
        img = env.render(mode='rgb_array')
        assert img is not None and img.shape == (1080, 1920, 3)
        env.render(mode='human', backend='null')
        assert env.viewer.shown == 1


def test_launch_env_flags():
    from blendtorch.btt.env import _flags
    assert _flags({'render_every': 10, 'real_time': False, 'x': True}) == \
        ['--render-every', '10', '--no-real-time', '--x']


def test_remote_env_timeout_is_valueerror(free_port):
    env = btt.env.RemoteEnv(f'tcp://127.0.0.1:{free_port}', timeoutms=100)
    with pytest.raises(ValueError, match='receive'):
        env.reset()
    env.close()


def test_env_registry_make_cartpole(free_port):
    """``btt.env.make`` resolves a registered id without gym (the reference
    relies on gym.make for blendtorch-cartpole-v0)."""
    import sys
    sys.path.insert(0, str(ROOT / 'examples' / 'control'))
    import cartpole_gym  # noqa: F401  registers the id
    from blendtorch import btt
    env = btt.env.make('blendtorch-cartpole-v0', launcher_args={'start_port': free_port})
    try:
        obs = env.reset()
        assert len(obs) == 3
        for _ in range(5):
            obs, reward, done, info = env.step(1.0)
        assert env.env_time is not None
    finally:
        env.close()
    with pytest.raises(KeyError):
        btt.env.make('no-such-env-v0')
