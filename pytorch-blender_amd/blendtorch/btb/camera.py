"""Camera intrinsics/extrinsics and world -> pixel projection.

API and numbers follow pkg_blender/blendtorch/btb/camera.py:8-204:
``view_matrix`` is the inverse of the camera's (scale-free) world matrix,
``proj_matrix`` Blender's ``calc_matrix_camera`` at the render size, and ::

    ndc   = dehom([p, 1] (P V)^T)
    pixel = (ndc.xy + 1) / 2 * [W, H]      (y mirrored for origin 'upper-left')
    depth = -([p, 1] V^T).z                (linear depth along the view axis)

All projections go through :func:`_project`, the same math as the batched
GPU path (:func:`blendtorch.ops.project` / ``ops.reference_project``).
"""
import bpy
import numpy as np
from mathutils import Vector

from . import utils

_ORIGINS = ('upper-left', 'lower-left')


def _as_np(m):
    return np.array(m, dtype=np.float64)


def _project(points, view, proj, want_depth):
    """Homogeneous projection of N x 3 points: (ndc N x 3, depth N or None)."""
    p = utils.hom(np.atleast_2d(np.asarray(points, dtype=np.float64)), 1.0)
    eye = p @ view.T                           # camera space
    ndc = utils.dehom(eye @ proj.T)
    return ndc, (-eye[:, 2] if want_depth else None)


def _render_shape(render=None):
    """(H, W) of the render output: resolution scaled by its percentage."""
    r = render if render is not None else bpy.context.scene.render
    pct = r.resolution_percentage / 100.0
    return int(r.resolution_y * pct), int(r.resolution_x * pct)


def _view_of(obj):
    """World -> camera transform of ``obj`` (scene camera if None)."""
    obj = obj if obj is not None else bpy.context.scene.camera
    return obj.matrix_world.normalized().inverted()


def _proj_of(obj, shape):
    """Camera -> clip transform of ``obj`` for an image of ``shape`` (H, W)."""
    obj = obj if obj is not None else bpy.context.scene.camera
    h, w = shape if shape is not None else _render_shape()
    return obj.calc_matrix_camera(bpy.context.evaluated_depsgraph_get(), x=w, y=h)


class Camera:
    """A Blender camera object (default: the scene camera) and its matrices.

    ``shape`` is (H, W) of the image the pixel coordinates refer to; it
    defaults to the scene's render size."""

    def __init__(self, bpy_camera=None, shape=None):
        self.bpy_camera = bpy_camera if bpy_camera is not None else bpy.context.scene.camera
        self.shape = tuple(shape) if shape is not None else _render_shape()
        self.update_view_matrix()
        self.update_proj_matrix()

    # -- matrices ----------------------------------------------------------------
    def update_view_matrix(self):
        """Re-read the extrinsics (after the camera moved)."""
        self.view_matrix = _view_of(self.bpy_camera)

    def update_proj_matrix(self):
        """Re-read the intrinsics (after lens / sensor / resolution changes)."""
        self.proj_matrix = _proj_of(self.bpy_camera, self.shape)

    # the reference exposes these as static methods of Camera
    shape_from_bpy = staticmethod(_render_shape)
    view_from_bpy = staticmethod(_view_of)
    proj_from_bpy = staticmethod(_proj_of)

    # -- properties ----------------------------------------------------------------
    @property
    def type(self):
        """Blender object type of the wrapped camera (as the reference); the
        projection kind is ``bpy_camera.data.type`` ('PERSP' / 'ORTHO')."""
        return self.bpy_camera.type

    @property
    def clip_range(self):
        """(near, far) clip distances."""
        d = self.bpy_camera.data
        return d.clip_start, d.clip_end

    # -- projection ----------------------------------------------------------------
    def world_to_ndc(self, xyz_world, return_depth=False):
        """N x 3 world points -> N x 3 normalised device coordinates, plus the
        N linear depths when ``return_depth``."""
        ndc, depth = _project(xyz_world, _as_np(self.view_matrix), _as_np(self.proj_matrix), return_depth)
        return (ndc, depth) if return_depth else ndc

    def ndc_to_pixel(self, ndc, origin='upper-left'):
        """NDC -> pixel coordinates with the origin at the image's 'upper-left'
        (OpenCV convention) or 'lower-left' (OpenGL) corner."""
        if origin not in _ORIGINS:
            raise AssertionError(f'origin must be one of {_ORIGINS}')
        h, w = self.shape
        uv = (np.atleast_2d(ndc)[:, :2] + 1.0) / 2.0
        if origin == _ORIGINS[0]:
            uv[:, 1] = 1.0 - uv[:, 1]
        return uv * np.array([[w, h]], dtype=np.float64)

    def _to_pixel(self, xyz, return_depth):
        ndc, depth = _project(xyz, _as_np(self.view_matrix), _as_np(self.proj_matrix), return_depth)
        px = self.ndc_to_pixel(ndc)
        return (px, depth) if return_depth else px

    def object_to_pixel(self, *objs, return_depth=False):
        """Pixel coordinates (and depths) of every mesh vertex of ``objs``."""
        return self._to_pixel(utils.world_coordinates(*objs), return_depth)

    def bbox_object_to_pixel(self, *objs, return_depth=False):
        """Pixel coordinates (and depths) of the 8 bounding-box corners of each of ``objs``."""
        return self._to_pixel(utils.bbox_world_coordinates(*objs), return_depth)

    def look_at(self, look_at=None, look_from=None):
        """Aim the camera's -Z axis at ``look_at`` (default: the origin) from
        ``look_from`` (default: where it is), keeping +Y up."""
        eye = Vector(look_from) if look_from is not None else Vector(self.bpy_camera.location)
        target = Vector(look_at) if look_at is not None else Vector((0.0, 0.0, 0.0))
        self.bpy_camera.rotation_euler = (target - eye).to_track_quat('-Z', 'Y').to_euler()
        self.bpy_camera.location = eye
        self.update_view_matrix()
