"""Remote (Blender-hosted) environments, gym style.

Reference: pkg_pytorch/blendtorch/btt/env.py.

* :class:`RemoteEnv` -- REQ client (LINGER 0, SNDTIMEO = 10 x timeout,
  RCVTIMEO = timeout, REQ_RELAXED + REQ_CORRELATE) on the native C++ client
  (round trip with the GIL released) or the Python socket API;
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
import pickle
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

# Environment registry: ``register``/``make`` mirror gym's, so examples can
# say ``btt.env.make('blendtorch-cartpole-v0')`` with or without gym (the
# reference relies on ``gym.make``, examples/control/cartpole_gym/__init__.py).
_REGISTRY = {}


def register(id, entry_point, **kwargs):
    """Register an env id -> ``'module:Class'`` (also with gym when installed)."""
    _REGISTRY[id] = (entry_point, dict(kwargs))
    if _gym is not None:
        try:
            _gym.envs.registration.register(id=id, entry_point=entry_point, kwargs=dict(kwargs))
        except Exception:  # already registered with gym
            pass


def make(id, **kwargs):
    """Instantiate a registered env (gym.make semantics for our own ids)."""
    if id not in _REGISTRY:
        if _gym is not None:
            return _gym.make(id, **kwargs)
        raise KeyError(f'no environment registered as {id!r}')
    entry_point, defaults = _REGISTRY[id]
    import importlib
    mod, _, attr = entry_point.partition(':')
    cls = getattr(importlib.import_module(mod), attr)
    return cls(**{**defaults, **kwargs})


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


class _SocketLink:
    """REQ client on the pyzmq-compatible transport: ``send``/``recv`` can be
    split so several envs overlap their round trips (VectorRemoteEnv's
    fallback path)."""

    def __init__(self, address, timeoutms):
        self.context = zmq.Context()
        self.socket = self.context.socket(zmq.REQ)
        opts = ((zmq.LINGER, 0), (zmq.SNDTIMEO, 10 * timeoutms), (zmq.RCVTIMEO, timeoutms),
                (zmq.REQ_RELAXED, 1), (zmq.REQ_CORRELATE, 1))
        for opt, value in opts:
            self.socket.setsockopt(opt, value)
        self.socket.connect(address)

    def send(self, request):
        try:
            self.socket.send_pyobj(request)
        except zmq.Again:
            raise ValueError('Failed to send to remote environment') from None

    def recv(self):
        try:
            return self.socket.recv_pyobj()
        except zmq.Again:
            raise ValueError('Failed to receive from remote environment') from None

    def roundtrip(self, request):
        self.send(request)
        return self.recv()

    def close(self):
        self.socket.close()


class _NativeLink:
    """The same REQ client in C++ (``_native.VecReq`` with one env): the
    whole round trip -- send, wait, receive -- runs with the GIL released."""

    def __init__(self, address, timeoutms):
        from .. import _native
        self._req = _native.VecReq([address], timeoutms, 1)

    def roundtrip(self, request):
        return pickle.loads(self._req.roundtrip(0, pickle.dumps(request, protocol=4)))

    def close(self):
        self._req.close()


class RemoteEnv:
    """Client of a remote ``btb.env.RemoteControlledAgent`` (gym-like).

    ``reset() -> (obs, info)`` and ``step(action) -> (obs, reward, done,
    info)``; every request carries the last remote ``time`` seen and a
    ``rgb_array`` in a reply is kept for :meth:`render`.  Timeouts raise
    ``ValueError``.  ``native=True`` (default when the native module is
    built) runs the round trip in C++; False uses the Python socket API."""

    def __init__(self, address, timeoutms=DEFAULT_TIMEOUTMS, native=True):
        self.env_time = None
        self.rgb_array = None
        self.viewer = None
        self._link = None
        if native:
            try:
                self._link = _NativeLink(address, timeoutms)
            except (ImportError, AttributeError):
                self._link = None
        if self._link is None:
            self._link = _SocketLink(address, timeoutms)

    def reset(self):
        """Restart the remote episode; returns ``(obs, info)``."""
        reply = self._request('reset')
        return reply.pop('obs'), reply

    def step(self, action):
        """Advance the remote simulation with ``action``."""
        reply = self._request('step', action=action)
        obs, reward, done = (reply.pop(k) for k in ('obs', 'reward', 'done'))
        return obs, reward, done, reply

    def render(self, mode='human', backend=None):
        """``'rgb_array'``: the last rendered frame (or None); ``'human'``:
        show it with a viewer from :mod:`~blendtorch.btt.env_rendering`."""
        frame = self.rgb_array
        if mode == 'rgb_array' or frame is None:
            return frame
        if self.viewer is None:
            self.viewer = create_renderer(backend)
        self.viewer.imshow(frame)

    def _request(self, cmd, **fields):
        return self._received(self._link.roundtrip(dict(cmd=cmd, time=self.env_time, **fields)))

    def _received(self, reply):
        self.env_time = reply['time']
        self.rgb_array = reply.pop('rgb_array', None)
        return reply

    # split request / reply (Python link only), so N envs can overlap
    def _send(self, **fields):
        self._link.send(dict(time=self.env_time, **fields))

    def _recv(self):
        return self._received(self._link.recv())

    def close(self):
        viewer, self.viewer = self.viewer, None
        if viewer is not None:
            viewer.close()
        link, self._link = self._link, None
        if link is not None:
            link.close()


@contextmanager
def launch_env(scene, script, background=False, producer=None, timeoutms=DEFAULT_TIMEOUTMS, launcher_args=None,
               **kwargs):
    """Launch one remote env instance and yield a connected :class:`RemoteEnv`.

    The instance gets a single named socket ``GYM``; remaining kwargs become
    the env script's command-line flags (``_flags``).  ``producer`` selects a
    headless stand-in (e.g. ``'cartpolesim'``) instead of Blender and
    ``launcher_args`` passes extra :class:`BlenderLauncher` arguments
    (``start_port``, ``proto``, ``blend_path``, ...).  Reference:
    pkg_pytorch/blendtorch/btt/env.py:135-189."""
    spec = dict(scene=scene, script=script, num_instances=1, named_sockets=['GYM'], instance_args=[_flags(kwargs)],
                background=background, producer=producer, **(launcher_args or {}))
    with ExitStack() as stack:
        launcher = stack.enter_context(BlenderLauncher(**spec))
        env = RemoteEnv(launcher.launch_info.addresses['GYM'][0], timeoutms=timeoutms)
        stack.callback(env.close)
        yield env


class OpenAIRemoteEnv(_GymEnv):
    """gym-style base of remote environments (old 4-tuple API; see
    examples/control/cartpole_gym).  :meth:`launch` starts the remote
    instance; the env owns it until :meth:`close`.  Reference:
    pkg_pytorch/blendtorch/btt/env.py:191-316."""

    metadata = {'render.modes': ['rgb_array', 'human']}

    def __init__(self, version='0.0.1'):
        self.__version__ = version
        self._stack = ExitStack()
        self._remote = None

    def launch(self, scene, script, background=False, **kwargs):
        """Start the remote environment (kwargs become script flags)."""
        if self._remote is not None:
            raise AssertionError('Environment already running.')
        self._remote = self._stack.enter_context(launch_env(scene=scene, script=script, background=background,
                                                            **kwargs))

    def _live(self):
        if self._remote is None:
            raise AssertionError('Environment not running.')
        return self._remote

    def step(self, action):
        return self._live().step(action)

    def reset(self):
        return self._live().reset()[0]

    def seed(self, seed):
        raise NotImplementedError('remote environments are seeded at launch (-btseed)')

    def render(self, mode='human'):
        return self._live().render(mode=mode)

    @property
    def env_time(self):
        return self._remote.env_time

    def close(self):
        stack, self._stack = self._stack, None
        self._remote = None
        if stack is not None:
            stack.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _PinnedStager:
    """Host -> device staging through pinned buffers that are never rewritten
    while a copy out of them may still be queued.

    A ``non_blocking`` H2D copy from pinned memory is only enqueued: if the
    stream is busy (a policy step in flight) the DMA runs later and reads
    whatever the buffer holds THEN.  Rewriting one buffer per step would let
    the device see the next step's observations.  Buffers rotate instead
    (``depth`` of them), and each is reused only after the event recorded
    behind its last copy has completed."""

    def __init__(self, depth=2):
        self.depth = depth
        self._slots = []          # [pinned tensor, event or None]
        self._next = 0

    def stage(self, arr, device, dtype):
        import torch
        arr = np.ascontiguousarray(arr)
        if not self._slots or tuple(self._slots[0][0].shape) != arr.shape or self._slots[0][0].dtype != dtype:
            self._slots = [[torch.empty(arr.shape, dtype=dtype).pin_memory(), None] for _ in range(self.depth)]
            self._next = 0
        slot = self._slots[self._next]
        self._next = (self._next + 1) % self.depth
        if slot[1] is not None:
            slot[1].synchronize()      # the copy that last read this buffer is done
        slot[0].numpy()[...] = arr
        out = slot[0].to(device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(device))
        slot[1] = ev
        return out


class VectorRemoteEnv:
    """N remote envs stepped concurrently; batched observations on a device.

    ``step(actions)`` sends all N requests before waiting for any reply, so
    the remote simulations advance in parallel and one round trip costs
    ~max(latency) instead of sum(latency).  The native client (C++, GIL
    released, numeric obs/reward/done decoded straight into arrays) is used
    for scalar actions and numeric observations of dimension ``obs_dim``;
    otherwise a Python fallback over :class:`RemoteEnv` is used.  Observations
    are packed into a pinned host buffer and copied to ``device`` with one
    non-blocking transfer.  ``infos(i)`` returns env i's full last reply.
    """

    def __init__(self, addresses, device=None, timeoutms=DEFAULT_TIMEOUTMS, obs_dim=None, native=True,
                 io_threads=0):
        self.addresses = list(addresses)
        self.device = device
        self.obs_dim = obs_dim
        self._obs_stager = _PinnedStager()
        self._rgb_stager = _PinnedStager()
        self._native = None
        self.envs = None
        if native:
            try:
                from .. import _native
                # io_threads 0: one native IO thread per 2 envs, at most 4
                self._native = _native.VecReq(self.addresses, timeoutms, io_threads)
            except (ImportError, AttributeError):
                self._native = None
        if self._native is None:
            self.envs = [RemoteEnv(a, timeoutms=timeoutms) for a in self.addresses]

    def __len__(self):
        return len(self.addresses)

    def _stage(self, obs):
        import torch
        arr = np.asarray(obs, dtype=np.float32)
        if self.device is None or torch.device(self.device).type == 'cpu':
            return torch.from_numpy(arr)
        return self._obs_stager.stage(arr, torch.device(self.device), torch.float32)

    def _exchange(self, which, cmd, actions):
        if self.obs_dim is None:   # discover the observation size once
            self._native.exchange(which[:1], cmd, np.asarray(actions[:1], np.float64), 0)
            r = self._native.last_reply(which[0])
            self.obs_dim = int(np.size(r.get('obs')))
            if len(which) == 1:
                o, rew, done = self._native.exchange([], cmd, np.zeros(0), self.obs_dim)
                obs = np.asarray(r['obs'], np.float64).reshape(1, -1)
                return obs, np.array([float(r.get('reward', 0.0))]), np.array([bool(r.get('done', False))])
            o, rew, done = self._native.exchange(which[1:], cmd, np.asarray(actions[1:], np.float64), self.obs_dim)
            first = np.asarray(r['obs'], np.float64).reshape(1, -1)
            return (np.concatenate([first, o]), np.concatenate([[float(r.get('reward', 0.0))], rew]),
                    np.concatenate([[bool(r.get('done', False))], done]))
        return self._native.exchange(which, cmd, np.asarray(actions, np.float64), self.obs_dim)

    def reset(self, which=None):
        """Reset all (or the listed) envs; returns (obs, replies-or-None)."""
        which = list(range(len(self))) if which is None else list(which)
        if self._native is not None:
            obs, _, _ = self._exchange(which, 'reset', np.zeros(len(which)))
            return self._stage(obs), None
        for i in which:
            self.envs[i]._send(cmd='reset')
        replies = [self.envs[i]._recv() for i in which]
        return self._stage([r.pop('obs') for r in replies]), replies

    def step(self, actions):
        """Step every env with its action; returns (obs, reward, done, replies-or-None)."""
        import torch
        if isinstance(actions, torch.Tensor):
            actions = actions.detach().cpu().numpy()
        actions = np.asarray(actions, dtype=np.float64).reshape(len(self), -1)[:, 0]
        if self._native is not None:
            obs, rew, done = self._exchange(list(range(len(self))), 'step', actions)
            return self._stage(obs), torch.from_numpy(np.asarray(rew)), torch.from_numpy(np.asarray(done)), None
        for e, a in zip(self.envs, actions):
            e._send(cmd='step', action=float(a))
        replies = [e._recv() for e in self.envs]
        obs = [r.pop('obs') for r in replies]
        rew = torch.tensor([float(r.pop('reward')) for r in replies])
        done = torch.tensor([bool(r.pop('done')) for r in replies])
        return self._stage(obs), rew, done, replies

    def step_async(self, actions):
        """Send every env its action and return at once (gym VectorEnv
        style): the remote simulations advance while the caller does other
        work (e.g. a training step); collect with :meth:`step_wait`."""
        import torch
        if self._native is None or self.obs_dim is None:
            self._async = actions          # Python path / first call: plain step in step_wait
            return
        if isinstance(actions, torch.Tensor):
            actions = actions.detach().cpu().numpy()
        actions = np.asarray(actions, dtype=np.float64).reshape(len(self), -1)[:, 0]
        self._native.exchange(list(range(len(self))), 'step', actions, self.obs_dim, 1)
        self._async = None

    def step_wait(self):
        """Replies to the last :meth:`step_async`: (obs, reward, done, replies-or-None)."""
        import torch
        pending = getattr(self, '_async', None)
        if pending is not None:
            self._async = None
            return self.step(pending)
        obs, rew, done = self._native.exchange(list(range(len(self))), 'step', np.zeros(0), self.obs_dim, 2)
        return self._stage(obs), torch.from_numpy(np.asarray(rew)), torch.from_numpy(np.asarray(done)), None

    def rgb_batch(self, decode=None, key='rgb_array'):
        """The latest rendered frames of all envs as one decoded GPU batch
        (pixel-based policies): the u8 ``HxWx3`` arrays of the last replies
        are packed into one pinned buffer, copied to ``device`` in a single
        transfer and run through the fused decode kernel (``decode``:
        :class:`~blendtorch.ops.DecodeConfig`, default /255 CHW fp32).
        Returns None when the envs did not render on their last step
        (``--render-every``)."""
        import torch
        from .. import ops
        replies = [self.infos(i) for i in range(len(self))] if self._native is not None else None
        if replies is None:
            raise NotImplementedError('rgb_batch needs the native client')
        frames = [r.get(key) for r in replies]
        if any(f is None for f in frames):
            return None
        arr = np.stack([np.asarray(f, dtype=np.uint8) for f in frames])
        decode = decode or ops.DecodeConfig.unit(channels='rgb')
        dev = torch.device(self.device) if self.device is not None else torch.device('cpu')
        if dev.type != 'cuda':
            return ops.reference_decode(torch.from_numpy(arr), decode)
        return ops.decode(self._rgb_stager.stage(arr, dev, torch.uint8), decode)

    def infos(self, i):
        """Full last reply of env i (native path) as a dict."""
        if self._native is not None:
            return self._native.last_reply(i)
        raise NotImplementedError('replies are returned by step() on the Python path')

    def close(self):
        if self._native is not None:
            self._native.close()
            self._native = None
        if self.envs:
            for e in self.envs:
                e.close()
            self.envs = None
