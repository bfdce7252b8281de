"""Blender-hosted environments and the remote-controlled agent.

Reference: pkg_blender/blendtorch/btb/env.py.

:class:`BaseEnv` lives inside the frame loop.  Each frame:

* ``pre_animation`` (first frame of an episode): state INIT,
  ``ctx = {'prev_action': None, 'done': False}``, ``_env_reset()``;
* ``pre_frame``: ``ctx['time'] = frame``; ``ctx['done'] |= frame >= end``;
  for frames after the first the agent is asked
  ``cmd, action = agent(env, **ctx)``; RESTART rewinds, STEP applies
  ``_env_prepare_step(action)`` (if not None) and records ``prev_action``;
* ``post_frame``: optional render into ``ctx['rgb_array']`` every n-th frame,
  then ``ctx.update(_env_post_step())``.

So the reply to request k is the state *after* the frame in which action k
was applied, sent at the next frame's pre_frame.  ``run`` plays up to frame
2147483647 so episodes may run past ``frame_range[1]`` (``done`` flags it).

:class:`RemoteControlledAgent` bridges this callback protocol to a remote
``btt.env.RemoteEnv`` over REQ/REP: a two-state (REQ/REP) machine, optional
``real_time`` mode (non-blocking; no request -> keep simulating without an
action), and the "reset while already INIT" short-circuit that answers the
reset immediately (``env.py:220-252``).
"""
import bpy

from ..transport import zmq
from .animation import AnimationController
from .camera import Camera
from .constants import DEFAULT_TIMEOUTMS
from .offscreen import OffScreenRenderer


class BaseEnv:
    """Abstract environment; implement ``_env_reset``, ``_env_prepare_step``
    and ``_env_post_step``."""

    STATE_INIT = object()
    STATE_RUN = object()
    CMD_RESTART = object()
    CMD_STEP = object()

    def __init__(self, agent):
        self.events = AnimationController()
        self.events.pre_frame.add(self._pre_frame)
        self.events.pre_animation.add(self._pre_animation)
        self.events.post_frame.add(self._post_frame)
        self.agent = agent
        self.ctx = None
        self.renderer = None
        self.render_every = None
        self.frame_range = None
        self.state = BaseEnv.STATE_INIT

    def run(self, frame_range=None, use_animation=True):
        """Hook into the frame loop and start playing."""
        self.frame_range = AnimationController.setup_frame_range(frame_range)
        self.events.play((self.frame_range[0], 2147483647), num_episodes=-1, use_animation=use_animation,
                         use_offline_render=True)

    def attach_default_renderer(self, every_nth=1):
        """Render the scene camera (rgb, gamma 2.2) into ``ctx['rgb_array']``
        every ``every_nth`` frame."""
        self.renderer = OffScreenRenderer(camera=Camera(), mode='rgb', gamma_coeff=2.2)
        self.render_every = every_nth

    def _pre_frame(self):
        frame = self.events.frameid
        self.ctx['time'] = frame
        self.ctx['done'] |= (frame >= self.frame_range[1])
        if frame > self.frame_range[0]:
            cmd, action = self.agent(self, **self.ctx)
            if cmd == BaseEnv.CMD_RESTART:
                self._restart()
            elif cmd == BaseEnv.CMD_STEP:
                if action is not None:
                    self._env_prepare_step(action)
                    self.ctx['prev_action'] = action
                self.state = BaseEnv.STATE_RUN

    def _pre_animation(self):
        self.state = BaseEnv.STATE_INIT
        self.ctx = {'prev_action': None, 'done': False}
        self._env_reset()

    def _post_frame(self):
        self._render(self.ctx)
        self.ctx = {**self.ctx, **self._env_post_step()}

    def _render(self, ctx):
        if self.renderer and ((self.events.frameid - self.frame_range[0]) % self.render_every) == 0:
            ctx['rgb_array'] = self.renderer.render()

    def _restart(self):
        self.events.rewind()

    def _env_reset(self):
        """Reset the environment state."""
        raise NotImplementedError()

    def _env_prepare_step(self, action):
        """Apply ``action`` before the frame is simulated."""
        raise NotImplementedError()

    def _env_post_step(self):
        """Return ``dict(obs=..., reward=..., [done=...], **info)`` after the frame."""
        raise NotImplementedError()


class RemoteControlledAgent:
    """Agent whose decisions come from a remote ``btt.env.RemoteEnv``."""

    STATE_REQ = 0
    STATE_REP = 1

    def __init__(self, address, real_time=False, timeoutms=DEFAULT_TIMEOUTMS):
        self.context = zmq.Context()
        self.socket = self.context.socket(zmq.REP)
        self.socket.setsockopt(zmq.LINGER, 0)
        self.socket.setsockopt(zmq.SNDTIMEO, timeoutms)
        self.socket.setsockopt(zmq.RCVTIMEO, timeoutms)
        self.socket.bind(address)
        self.real_time = real_time
        self.state = RemoteControlledAgent.STATE_REQ

    def __call__(self, env, **ctx):
        flags = zmq.NOBLOCK if (self.real_time and env.state == BaseEnv.STATE_RUN) else 0
        if self.state == RemoteControlledAgent.STATE_REP:
            try:
                self.socket.send_pyobj(ctx, flags=flags)
                self.state = RemoteControlledAgent.STATE_REQ
            except zmq.error.Again:
                if not self.real_time:
                    raise ValueError('Failed to send to remote agent.')
                return BaseEnv.CMD_STEP, None
        if self.state == RemoteControlledAgent.STATE_REQ:
            try:
                req = self.socket.recv_pyobj(flags=flags)
            except zmq.error.Again:
                return BaseEnv.CMD_STEP, None
            assert req['cmd'] in ['reset', 'step']
            self.state = RemoteControlledAgent.STATE_REP
            if req['cmd'] == 'reset':
                if env.state == BaseEnv.STATE_INIT:
                    # already at the start of an episode: answer right away
                    return self.__call__(env, **ctx)
                return BaseEnv.CMD_RESTART, None
            return BaseEnv.CMD_STEP, req['action']
