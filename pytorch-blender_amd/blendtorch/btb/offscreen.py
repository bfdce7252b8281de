"""Offscreen rendering of the scene through the first 3D view.

Contract (pkg_blender/blendtorch/btb/offscreen.py:9-112): the viewport
engine draws the scene with the camera's view/projection matrices into a
``gpu.types.GPUOffScreen(W, H)``; the colour texture is read back into a
reused u8 H x W x C buffer (C = 4 for ``'rgba'``, 3 for ``'rgb'``);
``origin='upper-left'`` flips GL's bottom-up rows; ``gamma_coeff`` applies
the reference's power law ``u8(255 * (x / 255) ** (1 / g))`` (float32 math,
truncation) to the colour channels and leaves alpha alone.

Readback: PyOpenGL's ``glGetTexImage`` where Blender still ships ``bgl``
(2.8x / 2.9x, as the reference), else the GPU module's
``texture_color.read()`` (newer Blender and the headless emulation).  The
gamma is a 256-entry table built once with the same float32 formula -- equal
to the per-pixel power law by construction and the same table the GPU decode
kernel uses (``blendtorch.ops.gamma_lut``).  Both the flip and the gamma can
instead be left to the consumer's decode kernel (``origin='lower-left'``
producer + ``btt.DecodeConfig(gamma=...)``).

Call :meth:`render` from ``post_frame`` (the AnimationController makes that
safe in interactive Blender).
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

_MODES = {'rgba': 4, 'rgb': 3}
_ORIGINS = ('upper-left', 'lower-left')


def _power_law_table(coeff):
    """u8[256]: the reference's gamma for every input byte (float32 math)."""
    x = np.arange(256, dtype=np.float32) / np.float32(255)
    return np.uint8(np.float32(255.0) * x ** np.float32(1.0 / coeff))


class OffScreenRenderer:
    """Render the scene as ``camera`` sees it into an H x W x C u8 array."""

    def __init__(self, camera=None, mode='rgba', origin='upper-left', gamma_coeff=None):
        if mode not in _MODES or origin not in _ORIGINS:
            raise AssertionError(f'mode must be in {tuple(_MODES)}, origin in {_ORIGINS}')
        self.camera = camera if camera is not None else Camera()
        self.origin, self.gamma_coeff = origin, gamma_coeff
        self.channels = _MODES[mode]
        h, w = self.shape
        self.offscreen = gpu.types.GPUOffScreen(w, h)
        self.area, self.space, self.region = find_first_view3d()
        self.handle = None
        self.buffer = np.zeros((h, w, self.channels), dtype=np.uint8)
        self._table = _power_law_table(gamma_coeff) if gamma_coeff else None
        use_gl = glGetTexImage is not None and bgl is not None and not getattr(bpy, '__headless__', False)
        self.mode = (bgl.GL_RGBA if mode == 'rgba' else bgl.GL_RGB) if bgl is not None else mode
        self._read = self._read_gl if use_gl else self._read_texture

    @property
    def shape(self):
        return self.camera.shape

    def _read_gl(self):
        bgl.glActiveTexture(bgl.GL_TEXTURE0)
        bgl.glBindTexture(bgl.GL_TEXTURE_2D, self.offscreen.color_texture)
        glGetTexImage(bgl.GL_TEXTURE_2D, 0, self.mode, bgl.GL_UNSIGNED_BYTE, self.buffer)

    def _read_texture(self):
        h, w = self.shape
        pixels = np.asarray(self.offscreen.texture_color.read(), dtype=np.uint8).reshape(h, w, -1)
        self.buffer[...] = pixels[..., :self.channels]

    def render(self):
        """Draw and read back one frame; returns the H x W x C u8 image."""
        with self.offscreen.bind():
            self.offscreen.draw_view3d(bpy.context.scene, bpy.context.view_layer, self.space, self.region,
                                       self.camera.view_matrix, self.camera.proj_matrix)
            self._read()
        img = self.buffer[::-1] if self.origin == _ORIGINS[0] else self.buffer
        return img if self._table is None else self._color_correct(img, self.gamma_coeff)

    def set_render_style(self, shading='RENDERED', overlays=False):
        """Viewport shading ('RENDERED', 'SOLID', ...) and overlay visibility."""
        self.space.shading.type = shading
        self.space.overlay.show_overlays = overlays

    def _color_correct(self, buffer, coeff=2.2):
        """Gamma on the colour channels through the 256-entry table."""
        table = self._table if (self._table is not None and coeff == self.gamma_coeff) else _power_law_table(coeff)
        out = np.array(buffer, dtype=np.uint8, copy=True)
        out[..., :3] = table[buffer[..., :3]]
        return out
