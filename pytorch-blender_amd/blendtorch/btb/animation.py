"""Blender frame loop with fine-grained callbacks.

Reference: pkg_blender/blendtorch/btb/animation.py:9-213.  Six signals:
``pre_play``, ``pre_animation``, ``pre_frame``, ``post_frame``,
``post_animation``, ``post_play``.  Two drivers:

* ``use_animation=True`` -- Blender's own (non-blocking, UI timer driven)
  playback: ``frame_change_pre`` drives pre-frame work and a POST_PIXEL draw
  handler of the first 3D view drives post-frame work, which makes offscreen
  rendering inside ``post_frame`` safe.  POST_PIXEL may fire several times
  per frame; a pending flag plus the last handled frame id suppresses
  duplicates (``:56-65``).
* ``use_animation=False`` -- a blocking ``frame_set`` loop (works with
  ``--background``), as fast as the scene evaluates.

``num_episodes=-1`` loops forever; ``rewind()`` restarts the episode; the
rigid-body cache range follows the animation range when ``use_physics``.
"""
import sys

import bpy

from .signal import Signal
from .utils import find_first_view3d


class AnimationController:
    """Drive Blender's animation system and emit per-frame signals."""

    def __init__(self):
        self.pre_animation = Signal()
        self.pre_frame = Signal()
        self.post_frame = Signal()
        self.post_animation = Signal()
        self.pre_play = Signal()
        self.post_play = Signal()
        self._plyctx = None

    class _PlayContext:
        """Book-keeping of one ``play`` call."""

        def __init__(self, frame_range, num_episodes, use_animation, use_offline_render):
            self.frame_range = frame_range
            self.num_episodes = num_episodes
            self.use_animation = use_animation
            self.use_offline_render = use_offline_render
            self.episode = 0
            self.pending_post_frame = False
            self.last_post_frame = 0
            self.draw_handler = None
            self.draw_space = None

        def skip_post_frame(self, current_frame):
            """True when a post-frame event must be ignored: nothing pending,
            already handled for this frame, or a redraw of another 3D view."""
            if not self.pending_post_frame or self.last_post_frame == current_frame:
                return True
            return (self.use_animation and self.use_offline_render
                    and bpy.context.space_data != self.draw_space)

    @property
    def frameid(self):
        """Current frame number of the scene."""
        return bpy.context.scene.frame_current

    def play(self, frame_range=None, num_episodes=-1, use_animation=True, use_offline_render=True,
             use_physics=True):
        """Start playing ``frame_range`` (inclusive) ``num_episodes`` times."""
        assert self._plyctx is None, 'Animation already running'
        self._plyctx = AnimationController._PlayContext(
            frame_range=AnimationController.setup_frame_range(frame_range, physics=use_physics),
            num_episodes=num_episodes if num_episodes >= 0 else sys.maxsize,
            use_animation=use_animation,
            use_offline_render=use_offline_render)
        if use_animation:
            self._play_animation()
        else:
            self._play_manual()

    @staticmethod
    def setup_frame_range(frame_range, physics=True):
        """Apply ``frame_range`` (or the scene's) to the scene and, with
        ``physics``, to the rigid-body point cache; returns the range."""
        scene = bpy.context.scene
        if frame_range is None:
            frame_range = (scene.frame_start, scene.frame_end)
        scene.frame_start, scene.frame_end = frame_range[0], frame_range[1]
        if physics and scene.rigidbody_world:
            scene.rigidbody_world.point_cache.frame_start = frame_range[0]
            scene.rigidbody_world.point_cache.frame_end = frame_range[1]
        return frame_range

    def _play_animation(self):
        self.pre_play.invoke()
        bpy.app.handlers.frame_change_pre.append(self._on_pre_frame)
        if self._plyctx.use_offline_render:
            _, self._plyctx.draw_space, _ = find_first_view3d()
            self._plyctx.draw_handler = bpy.types.SpaceView3D.draw_handler_add(
                self._on_post_frame, (), 'WINDOW', 'POST_PIXEL')
        else:
            bpy.app.handlers.frame_change_post.append(self._on_post_frame)
        bpy.context.scene.frame_set(self._plyctx.frame_range[0])
        bpy.ops.screen.animation_play()   # returns immediately

    def _play_manual(self):
        self.pre_play.invoke()
        bpy.app.handlers.frame_change_pre.append(self._on_pre_frame)
        bpy.app.handlers.frame_change_post.append(self._on_post_frame)
        ctx = self._plyctx
        while ctx.episode < ctx.num_episodes:
            bpy.context.scene.frame_set(ctx.frame_range[0])
            while self.frameid < ctx.frame_range[1]:
                bpy.context.scene.frame_set(self.frameid + 1)
                if self._plyctx is None:   # _cancel ran inside frame_set
                    return

    def rewind(self):
        """Jump back to the first frame of the range (starts a new episode)."""
        if self._plyctx is not None:
            self._set_frame(self._plyctx.frame_range[0])

    def _set_frame(self, frame_index):
        bpy.context.scene.frame_set(frame_index)

    def _on_pre_frame(self, scene, *args):
        if self.frameid == self._plyctx.frame_range[0]:
            self.pre_animation.invoke()
        self.pre_frame.invoke()
        self._plyctx.pending_post_frame = True

    def _on_post_frame(self, *args):
        ctx = self._plyctx
        if ctx is None or ctx.skip_post_frame(self.frameid):
            return
        ctx.pending_post_frame = False
        ctx.last_post_frame = self.frameid
        self.post_frame.invoke()
        if self.frameid == ctx.frame_range[1]:
            self.post_animation.invoke()
            ctx.episode += 1
            if ctx.episode == ctx.num_episodes:
                self._cancel()

    def _cancel(self):
        bpy.app.handlers.frame_change_pre.remove(self._on_pre_frame)
        if self._plyctx.draw_handler is not None:
            bpy.types.SpaceView3D.draw_handler_remove(self._plyctx.draw_handler, 'WINDOW')
            self._plyctx.draw_handler = None
        else:
            bpy.app.handlers.frame_change_post.remove(self._on_post_frame)
        bpy.ops.screen.animation_cancel(restore_frame=False)
        self.post_play.invoke()
        self._plyctx = None
