"""Blender frame loop with fine-grained callbacks.

Behavioural contract (reference: pkg_blender/blendtorch/btb/animation.py:9-213):
six :class:`~blendtorch.btb.signal.Signal` s fire in this order for a range
``(a, b)`` and E episodes ::

    pre_play
    E x [ pre_animation, (pre_frame, post_frame) for a..b, post_animation ]
    post_play

Two ways of advancing frames:

* ``use_animation=True`` (interactive Blender): Blender's timer-driven
  playback runs the frames and :meth:`play` returns at once.  Frame changes
  arrive through ``frame_change_pre``; post-frame work is attached to the
  first 3D view's POST_PIXEL draw callback (``use_offline_render``), because
  only inside a draw callback may an offscreen render read the GL context.
  A view may be drawn several times per frame and other views draw too, so a
  post-frame event is accepted once per frame and only from that view.
* ``use_animation=False`` (``--background``): :meth:`play` itself steps
  ``frame_set`` through the range, as fast as the scene evaluates.

``num_episodes=-1`` plays forever; :meth:`rewind` jumps back to the first
frame (a new episode starts there); with ``use_physics`` the rigid-body point
cache is resized to the range so simulations run over all of it.
"""
import sys

import bpy

from .signal import Signal
from .utils import find_first_view3d

_SIGNALS = ('pre_play', 'pre_animation', 'pre_frame', 'post_frame', 'post_animation', 'post_play')


class _Run:
    """State of one :meth:`AnimationController.play` call."""

    __slots__ = ('first', 'last', 'episodes_left', 'timer_driven', 'draw_bound', 'awaiting_post', 'posted_frame',
                 'view_space', 'draw_handle')

    def __init__(self, first, last, episodes, timer_driven, draw_bound):
        self.first, self.last = first, last
        self.episodes_left = episodes
        self.timer_driven = timer_driven
        self.draw_bound = draw_bound          # post-frame work runs in a 3D view's draw callback
        self.awaiting_post = False            # a pre-frame fired and its post-frame has not run yet
        self.posted_frame = None              # frame whose post-frame already ran
        self.view_space = None
        self.draw_handle = None

    def accepts_post(self, frame):
        """One post-frame event per frame, and (draw-bound) only from our view."""
        if not self.awaiting_post or self.posted_frame == frame:
            return False
        if self.draw_bound and bpy.context.space_data != self.view_space:
            return False
        return True


class AnimationController:
    """Drive Blender's animation system and emit per-frame signals
    (``pre_play``, ``pre_animation``, ``pre_frame``, ``post_frame``,
    ``post_animation``, ``post_play``)."""

    def __init__(self):
        for name in _SIGNALS:
            setattr(self, name, Signal())
        self._run = None

    @property
    def frameid(self):
        """Current frame number of the scene."""
        return bpy.context.scene.frame_current

    @staticmethod
    def setup_frame_range(frame_range, physics=True):
        """Make ``frame_range`` (default: the scene's) the scene's range and,
        with ``physics``, the rigid-body cache's range.  Returns ``(a, b)``."""
        scene = bpy.context.scene
        first, last = frame_range if frame_range is not None else (scene.frame_start, scene.frame_end)
        scene.frame_start, scene.frame_end = first, last
        world = scene.rigidbody_world if physics else None
        if world:
            cache = world.point_cache
            cache.frame_start, cache.frame_end = first, last
        return (first, last)

    def play(self, frame_range=None, num_episodes=-1, use_animation=True, use_offline_render=True,
             use_physics=True):
        """Play ``frame_range`` (inclusive) ``num_episodes`` times (-1: forever).

        Blocking unless ``use_animation`` (then Blender's timer drives frames)."""
        if self._run is not None:
            raise AssertionError('Animation already running')
        first, last = self.setup_frame_range(frame_range, physics=use_physics)
        episodes = sys.maxsize if num_episodes < 0 else num_episodes
        self._run = run = _Run(first, last, episodes, use_animation, use_animation and use_offline_render)
        self.pre_play.invoke()
        bpy.app.handlers.frame_change_pre.append(self._frame_begins)
        if run.draw_bound:
            _, run.view_space, _ = find_first_view3d()
            run.draw_handle = bpy.types.SpaceView3D.draw_handler_add(self._frame_ends, (), 'WINDOW', 'POST_PIXEL')
        else:
            bpy.app.handlers.frame_change_post.append(self._frame_ends)
        if use_animation:
            bpy.context.scene.frame_set(first)
            bpy.ops.screen.animation_play()       # returns immediately; the timer takes over
            return
        scene = bpy.context.scene
        while self._run is run:
            scene.frame_set(first)
            while self._run is run and scene.frame_current < last:
                scene.frame_set(scene.frame_current + 1)

    def rewind(self):
        """Jump back to the first frame of the range (starts a new episode)."""
        if self._run is not None:
            bpy.context.scene.frame_set(self._run.first)

    # -- handlers --------------------------------------------------------------
    def _frame_begins(self, scene, *unused):
        run = self._run
        if self.frameid == run.first:
            self.pre_animation.invoke()
        self.pre_frame.invoke()
        run.awaiting_post = True

    def _frame_ends(self, *unused):
        run = self._run
        frame = self.frameid
        if run is None or not run.accepts_post(frame):
            return
        run.awaiting_post = False
        run.posted_frame = frame
        self.post_frame.invoke()
        if frame != run.last:
            return
        self.post_animation.invoke()
        run.episodes_left -= 1
        if run.episodes_left == 0:
            self._finish()

    def _finish(self):
        run = self._run
        bpy.app.handlers.frame_change_pre.remove(self._frame_begins)
        if run.draw_handle is not None:
            bpy.types.SpaceView3D.draw_handler_remove(run.draw_handle, 'WINDOW')
        else:
            bpy.app.handlers.frame_change_post.remove(self._frame_ends)
        bpy.ops.screen.animation_cancel(restore_frame=False)
        self._run = None
        self.post_play.invoke()
