"""Offscreen rendering of the scene through the first 3D view.

Reference: pkg_blender/blendtorch/btb/offscreen.py:9-112.  Renders with the
viewport engine into ``gpu.types.GPUOffScreen(W, H)`` using the camera's
view/projection matrices and reads the colour texture back into a reused
u8 HxWxC buffer; ``origin='upper-left'`` flips the GL (bottom-up) image;
optional gamma ``u8(255 * (x/255)**(1/g))`` on RGB, alpha untouched.

Readback uses PyOpenGL's ``glGetTexImage`` when available (Blender 2.8x/2.9x,
as the reference) and the GPU module's ``texture_color.read()`` otherwise
(newer Blender, and the headless emulation).

Call :meth:`render` from ``post_frame`` (AnimationController makes that
safe).  Gamma/flip can also be deferred to the GPU decode kernel on the
consumer side (``origin='lower-left'`` producer + ``btt.DecodeConfig``).
"""
import bpy
import gpu
import numpy as np

from .camera import Camera
from .utils import find_first_view3d

try:
    import bgl
except ImportError:  # Blender >= 4 removed bgl
    bgl = None
try:
    from OpenGL.GL import glGetTexImage
except ImportError:
    glGetTexImage = None


class OffScreenRenderer:
    """Render the scene as the camera sees it; ``mode`` 'rgba' or 'rgb'."""

    def __init__(self, camera=None, mode='rgba', origin='upper-left', gamma_coeff=None):
        assert mode in ['rgba', 'rgb']
        assert origin in ['upper-left', 'lower-left']
        self.camera = camera or Camera()
        self.offscreen = gpu.types.GPUOffScreen(self.shape[1], self.shape[0])
        self.area, self.space, self.region = find_first_view3d()
        self.handle = None
        self.origin = origin
        self.gamma_coeff = gamma_coeff
        self.channels = 4 if mode == 'rgba' else 3
        self.buffer = np.zeros((self.shape[0], self.shape[1], self.channels), dtype=np.uint8)
        self.mode = (bgl.GL_RGBA if mode == 'rgba' else bgl.GL_RGB) if bgl is not None else mode

    @property
    def shape(self):
        return self.camera.shape

    def render(self):
        """Render and return the HxWxC u8 image (C = 4 for rgba, 3 for rgb)."""
        with self.offscreen.bind():
            self.offscreen.draw_view3d(bpy.context.scene, bpy.context.view_layer, self.space, self.region,
                                       self.camera.view_matrix, self.camera.proj_matrix)
            if glGetTexImage is not None and bgl is not None and not getattr(bpy, '__headless__', False):
                bgl.glActiveTexture(bgl.GL_TEXTURE0)
                bgl.glBindTexture(bgl.GL_TEXTURE_2D, self.offscreen.color_texture)
                glGetTexImage(bgl.GL_TEXTURE_2D, 0, self.mode, bgl.GL_UNSIGNED_BYTE, self.buffer)
            else:
                rgba = np.asarray(self.offscreen.texture_color.read(), dtype=np.uint8)
                self.buffer[...] = rgba.reshape(self.shape[0], self.shape[1], -1)[..., :self.channels]
        buf = self.buffer
        if self.origin == 'upper-left':
            buf = np.flipud(buf)
        if self.gamma_coeff:
            buf = self._color_correct(buf, self.gamma_coeff)
        return buf

    def set_render_style(self, shading='RENDERED', overlays=False):
        self.space.shading.type = shading
        self.space.overlay.show_overlays = overlays

    def _color_correct(self, buffer, coeff=2.2):
        """Power-law gamma on RGB with float32 math + truncation (bit-exact with
        the reference and with the GPU decode kernel's LUT)."""
        rgb = buffer[..., :3].astype(np.float32) / 255
        rgb = np.uint8(255.0 * rgb ** (1 / coeff))
        if buffer.shape[-1] == 4:
            return np.concatenate((rgb, buffer[..., 3:4]), axis=-1)
        return rgb
