"""Blender-hosted environments and the remote-controlled agent.

Protocol (reference: pkg_blender/blendtorch/btb/env.py:10-252, pinned by
tests/test_env.py):

* an episode starts on its first frame: ``ctx = {'prev_action': None,
  'done': False}``, ``_env_reset()``, state INIT;
* before every frame: ``ctx['time']`` is the frame, ``ctx['done']`` latches
  once the frame reaches the range's end; from the second frame on the agent
  decides ``cmd, action = agent(env, **ctx)`` -- RESTART rewinds the
  animation, STEP applies ``_env_prepare_step(action)`` (when an action came)
  and the state becomes RUN;
* after every frame: every n-th frame is rendered into ``ctx['rgb_array']``
  and ``_env_post_step()``'s dict is merged into ``ctx``.

Hence the reply to request k is the state AFTER the frame that applied
action k, sent from the NEXT frame's pre-frame hook.  :meth:`BaseEnv.run`
plays to frame 2147483647 so an episode can run past the nominal end (the
``done`` flag reports it).

:class:`RemoteControlledAgent` answers a ``btt.env.RemoteEnv`` over REQ/REP.
"""

from ..transport import zmq
from . import animation, camera, constants, offscreen

_LAST_FRAME = 2147483647


def _rep_socket(address, timeoutms):
    """Bound REP socket with the reference's options (no linger, send and
    receive timeouts)."""
    ctx = zmq.Context()
    sock = ctx.socket(zmq.REP)
    for opt, value in ((zmq.LINGER, 0), (zmq.SNDTIMEO, timeoutms), (zmq.RCVTIMEO, timeoutms)):
        sock.setsockopt(opt, value)
    sock.bind(address)
    return ctx, sock


class BaseEnv:
    """Environment living in Blender's frame loop.

    Subclasses implement ``_env_reset()``, ``_env_prepare_step(action)`` and
    ``_env_post_step() -> dict(obs=..., reward=..., [done=...], **info)``."""

    STATE_INIT = object()
    STATE_RUN = object()
    CMD_RESTART = object()
    CMD_STEP = object()

    def __init__(self, agent):
        self.agent, self.events = agent, animation.AnimationController()
        self.ctx = self.frame_range = self.renderer = self.render_every = None
        self.state = self.STATE_INIT
        for signal, hook in (('pre_animation', self._episode_begins), ('pre_frame', self._before_frame),
                             ('post_frame', self._after_frame)):
            getattr(self.events, signal).add(hook)

    def run(self, frame_range=None, use_animation=True):
        """Attach to the frame loop and play.  ``use_animation=False`` is the
        blocking loop (``--background``, fastest); True keeps the UI live."""
        first, last = animation.AnimationController.setup_frame_range(frame_range)
        self.frame_range = (first, last)
        self.events.play((first, _LAST_FRAME), num_episodes=-1, use_animation=use_animation,
                         use_offline_render=True)

    def attach_default_renderer(self, every_nth=1):
        """Render the scene camera (RGB, gamma 2.2) into ``ctx['rgb_array']``
        on every ``every_nth`` frame (``env.render()`` on the remote side)."""
        self.renderer, self.render_every = (offscreen.OffScreenRenderer(camera=camera.Camera(), mode='rgb',
                                                                        gamma_coeff=2.2), every_nth)

    # -- frame-loop hooks --------------------------------------------------------
    def _episode_begins(self):
        self.ctx, self.state = dict(prev_action=None, done=False), self.STATE_INIT
        self._env_reset()

    def _before_frame(self):
        first, last = self.frame_range
        now = self.events.frameid
        self.ctx['time'] = now
        if now >= last:
            self.ctx['done'] = True
        if now <= first:
            return                          # the episode's first frame needs no decision
        command, action = self.agent(self, **self.ctx)
        if command is self.CMD_RESTART:
            self.events.rewind()
        elif command is self.CMD_STEP:
            if action is not None:
                self._env_prepare_step(action)
                self.ctx.update(prev_action=action)
            self.state = self.STATE_RUN

    def _after_frame(self):
        if self.renderer is not None and (self.events.frameid - self.frame_range[0]) % self.render_every == 0:
            self.ctx['rgb_array'] = self.renderer.render()
        self.ctx.update(self._env_post_step())

    # -- to implement ------------------------------------------------------------
    def _env_reset(self):
        """Bring the scene to the start state of an episode."""
        raise NotImplementedError(f'{type(self).__name__}._env_reset')

    def _env_prepare_step(self, action):
        """Apply ``action`` before the frame is simulated."""
        raise NotImplementedError(f'{type(self).__name__}._env_prepare_step')

    def _env_post_step(self):
        """Observation, reward, optional done flag and extras after the frame."""
        raise NotImplementedError(f'{type(self).__name__}._env_post_step')


class RemoteControlledAgent:
    """Agent whose decisions come from a remote ``btt.env.RemoteEnv``.

    A REP socket (bound at ``address``) alternates between awaiting a request
    (STATE_REQ) and owing its reply (STATE_REP); the reply to a request is the
    ctx of the next frame.  ``real_time``: while the episode runs, the socket
    is polled without blocking and a frame without a request simply advances
    the simulation (no action) -- the scene does not wait for the agent.  A
    receive timeout does the same in the blocking mode; a send that times out
    there is an error."""

    STATE_REQ = 0
    STATE_REP = 1

    def __init__(self, address, real_time=False, timeoutms=constants.DEFAULT_TIMEOUTMS):
        self.context, self.socket = _rep_socket(address, timeoutms)
        self.real_time, self.state = real_time, self.STATE_REQ

    def __call__(self, env, **ctx):
        flags = zmq.NOBLOCK if (self.real_time and env.state is env.STATE_RUN) else 0
        keep_going = (BaseEnv.CMD_STEP, None)     # simulate the frame without an action
        if self.state == self.STATE_REP and not self._reply(ctx, flags):
            return keep_going
        try:
            request = self.socket.recv_pyobj(flags=flags)
        except zmq.Again:
            return keep_going                      # nobody asked in time
        cmd = request['cmd']
        assert cmd in ('reset', 'step'), f'unknown command {cmd!r}'
        self.state = self.STATE_REP
        if cmd == 'step':
            return BaseEnv.CMD_STEP, request['action']
        if env.state is env.STATE_INIT:
            # already at an episode's start: the current ctx IS the reset state
            return self(env, **ctx)
        return BaseEnv.CMD_RESTART, None

    def _reply(self, ctx, flags):
        """Send the owed reply; False when it could not go out in real-time mode."""
        try:
            self.socket.send_pyobj(ctx, flags=flags)
        except zmq.Again:
            if self.real_time:
                return False
            raise ValueError('Failed to send the reply to the remote agent.') from None
        self.state = self.STATE_REQ
        return True
