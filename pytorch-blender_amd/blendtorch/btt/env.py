"""Remote (Blender-hosted) environments, gym style.

Reference: pkg_pytorch/blendtorch/btt/env.py.

* :class:`RemoteEnv` -- REQ socket that connects (LINGER 0, SNDTIMEO =
  10 x timeout, RCVTIMEO = timeout, REQ_RELAXED + REQ_CORRELATE);
  ``reset() -> (obs, info)``, ``step(a) -> (obs, reward, done, info)``;
  every request carries the last seen remote ``time``; send/receive timeouts
  surface as ``ValueError`` (``env.py:34-133``).
* :func:`launch_env` -- launches one instance with a ``GYM`` socket and
  yields a RemoteEnv; kwargs become ``--key value`` / ``--key`` /
  ``--no-key`` flags (``env.py:135-189``).
* :class:`OpenAIRemoteEnv` -- gym.Env base (old 4-tuple API).  The reference
  defines it only when gym imports; here it always exists and derives from
  ``gym.Env`` when gym is installed, else from a minimal compatible base.
* :class:`VectorRemoteEnv` (new) -- steps N remote envs concurrently
  (requests fanned out, replies gathered) and stages the batched
  observations in device memory for a GPU policy.
"""
from contextlib import ExitStack, contextmanager

import numpy as np

from ..transport import zmq
from .constants import DEFAULT_TIMEOUTMS
from .env_rendering import create_renderer
from .launcher import BlenderLauncher

try:  # optional dependency, as in the reference
    import gym as _gym
    _GymEnv = _gym.Env
except ImportError:  # pragma: no cover - gym is not in this image
    _gym = None

    class _GymEnv:
        """Minimal stand-in for ``gym.Env`` (metadata, reward_range, spaces)."""
        metadata = {'render.modes': []}
        reward_range = (-float('inf'), float('inf'))
        action_space = None
        observation_space = None

        def close(self):
            pass

        @property
        def unwrapped(self):
            return self

GYM_AVAILABLE = _gym is not None


def _flags(kwargs):
    """``launch_env`` kwargs -> argparse-style command-line flags."""
    args = []
    for k, v in kwargs.items():
        k = k.replace('_', '-')
        if isinstance(v, bool):
            args.append(f'--{k}' if v else f'--no-{k}')
        else:
            args.extend([f'--{k}', str(v)])
    return args


class RemoteEnv:
    """Client of a remote ``btb.env.RemoteControlledAgent``."""

    def __init__(self, address, timeoutms=DEFAULT_TIMEOUTMS):
        self.context = zmq.Context()
        self.socket = self.context.socket(zmq.REQ)
        self.socket.setsockopt(zmq.LINGER, 0)
        self.socket.setsockopt(zmq.SNDTIMEO, timeoutms * 10)
        self.socket.setsockopt(zmq.RCVTIMEO, timeoutms)
        self.socket.setsockopt(zmq.REQ_RELAXED, 1)
        self.socket.setsockopt(zmq.REQ_CORRELATE, 1)
        self.socket.connect(address)
        self.env_time = None
        self.rgb_array = None
        self.viewer = None

    def reset(self):
        """Reset the remote env; returns ``(obs, info)``."""
        d = self._reqrep(cmd='reset')
        self.rgb_array = d.pop('rgb_array', None)
        return d.pop('obs'), d

    def step(self, action):
        """Apply ``action``; returns ``(obs, reward, done, info)``."""
        d = self._reqrep(cmd='step', action=action)
        obs = d.pop('obs')
        reward = d.pop('reward')
        done = d.pop('done')
        self.rgb_array = d.pop('rgb_array', None)
        return obs, reward, done, d

    def render(self, mode='human', backend=None):
        """Return (``rgb_array``) or show (``human``) the last remote frame."""
        if mode == 'rgb_array' or self.rgb_array is None:
            return self.rgb_array
        if self.viewer is None:
            self.viewer = create_renderer(backend)
        self.viewer.imshow(self.rgb_array)

    # split request/reply so many envs can be stepped concurrently
    def _send(self, **kw):
        try:
            self.socket.send_pyobj({**kw, 'time': self.env_time})
        except zmq.error.Again:
            raise ValueError('Failed to send to remote environment') from None

    def _recv(self):
        try:
            d = self.socket.recv_pyobj()
        except zmq.error.Again:
            raise ValueError('Failed to receive from remote environment') from None
        self.env_time = d['time']
        return d

    def _reqrep(self, **send_kwargs):
        self._send(**send_kwargs)
        return self._recv()

    def close(self):
        if self.viewer:
            self.viewer.close()
            self.viewer = None
        if self.socket:
            self.socket.close()
            self.socket = None


@contextmanager
def launch_env(scene, script, background=False, producer=None, timeoutms=DEFAULT_TIMEOUTMS, **kwargs):
    """Launch one remote env instance and yield a connected :class:`RemoteEnv`.

    ``producer`` selects a headless stand-in (e.g. ``'cartpolesim'``) instead
    of Blender; remaining kwargs become command-line flags of the env script.
    """
    env = None
    try:
        launch = dict(scene=scene, script=script, num_instances=1, named_sockets=['GYM'],
                      instance_args=[_flags(kwargs)], background=background, producer=producer)
        with BlenderLauncher(**launch) as bl:
            env = RemoteEnv(bl.launch_info.addresses['GYM'][0], timeoutms=timeoutms)
            yield env
    finally:
        if env:
            env.close()


class OpenAIRemoteEnv(_GymEnv):
    """Base class of gym-registered remote environments (see
    examples/control/cartpole_gym)."""

    metadata = {'render.modes': ['rgb_array', 'human']}

    def __init__(self, version='0.0.1'):
        self.__version__ = version
        self._es = ExitStack()
        self._env = None

    def launch(self, scene, script, background=False, **kwargs):
        """Launch the remote environment (kwargs -> command-line flags)."""
        assert not self._env, 'Environment already running.'
        self._env = self._es.enter_context(launch_env(scene=scene, script=script, background=background, **kwargs))

    def step(self, action):
        assert self._env, 'Environment not running.'
        obs, reward, done, info = self._env.step(action)
        return obs, reward, done, info

    def reset(self):
        assert self._env, 'Environment not running.'
        obs, info = self._env.reset()
        return obs

    def seed(self, seed):
        raise NotImplementedError()

    def render(self, mode='human'):
        assert self._env, 'Environment not running.'
        return self._env.render(mode=mode)

    @property
    def env_time(self):
        return self._env.env_time

    def close(self):
        if self._es:
            self._es.close()
            self._es = None
            self._env = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class VectorRemoteEnv:
    """N remote envs stepped concurrently; batched observations on a device.

    ``step(actions)`` sends all N requests before waiting for any reply, so
    the remote simulations advance in parallel and one round trip costs
    ~max(latency) instead of sum(latency).  Observations (numeric tuples /
    arrays) are packed into a pinned host buffer and copied to ``device``
    with one non-blocking transfer; rewards/dones come back as tensors too.
    """

    def __init__(self, addresses, device=None, timeoutms=DEFAULT_TIMEOUTMS):
        self.envs = [RemoteEnv(a, timeoutms=timeoutms) for a in addresses]
        self.device = device
        self._pinned = None

    def __len__(self):
        return len(self.envs)

    def _stage(self, obs):
        import torch
        arr = np.asarray(obs, dtype=np.float32)
        if self.device is None or torch.device(self.device).type == 'cpu':
            return torch.from_numpy(arr)
        if self._pinned is None or tuple(self._pinned.shape) != arr.shape:
            self._pinned = torch.empty(arr.shape, dtype=torch.float32).pin_memory()
        self._pinned.numpy()[...] = arr
        return self._pinned.to(self.device, non_blocking=True)

    def reset(self):
        for e in self.envs:
            e._send(cmd='reset')
        replies = [e._recv() for e in self.envs]
        obs = [r.pop('obs') for r in replies]
        return self._stage(obs), replies

    def step(self, actions):
        import torch
        if isinstance(actions, torch.Tensor):
            actions = actions.detach().cpu().numpy()
        for e, a in zip(self.envs, actions):
            e._send(cmd='step', action=a.item() if hasattr(a, 'item') else a)
        replies = [e._recv() for e in self.envs]
        obs = [r.pop('obs') for r in replies]
        rew = torch.tensor([float(r.pop('reward')) for r in replies])
        done = torch.tensor([bool(r.pop('done')) for r in replies])
        return self._stage(obs), rew, done, replies

    def close(self):
        for e in self.envs:
            e.close()
