"""Camera intrinsics/extrinsics and world->pixel projection.

Reference: pkg_blender/blendtorch/btb/camera.py:8-204.  ``view_matrix`` is
the inverse of the camera's normalised world matrix, ``proj_matrix`` comes
from ``calc_matrix_camera`` at the render resolution.  Projection:

    ndc   = dehom([p, 1] @ (P V)^T)
    pixel = ((ndc.xy + 1) / 2) * [W, H]   (y flipped for 'upper-left')
    depth = -([p, 1] @ V^T).z             (linear camera-space depth)

For many points at once on the GPU see :func:`blendtorch.ops.project`.
"""
import bpy
import numpy as np
from mathutils import Vector

from . import utils


class Camera:
    """Thin wrapper of a Blender camera object (scene camera by default)."""

    def __init__(self, bpy_camera=None, shape=None):
        self.bpy_camera = bpy_camera or bpy.context.scene.camera
        self.shape = shape or Camera.shape_from_bpy()
        self.view_matrix = Camera.view_from_bpy(self.bpy_camera)
        self.proj_matrix = Camera.proj_from_bpy(self.bpy_camera, self.shape)

    def update_view_matrix(self):
        self.view_matrix = Camera.view_from_bpy(self.bpy_camera)

    def update_proj_matrix(self):
        self.proj_matrix = Camera.proj_from_bpy(self.bpy_camera, self.shape)

    @property
    def type(self):
        """Blender type of the wrapped object (as the reference: ``bpy_camera.type``);
        the projection kind is ``bpy_camera.data.type`` ('PERSP' / 'ORTHO')."""
        return self.bpy_camera.type

    @property
    def clip_range(self):
        return (self.bpy_camera.data.clip_start, self.bpy_camera.data.clip_end)

    @staticmethod
    def shape_from_bpy(bpy_render=None):
        """(H, W) of the render output (resolution x percentage)."""
        render = bpy_render or bpy.context.scene.render
        s = render.resolution_percentage / 100.0
        return (int(render.resolution_y * s), int(render.resolution_x * s))

    @staticmethod
    def view_from_bpy(bpy_camera):
        camera = bpy_camera or bpy.context.scene.camera
        return camera.matrix_world.normalized().inverted()

    @staticmethod
    def proj_from_bpy(bpy_camera, shape):
        camera = bpy_camera or bpy.context.scene.camera
        shape = shape or Camera.shape_from_bpy()
        return camera.calc_matrix_camera(bpy.context.evaluated_depsgraph_get(), x=shape[1], y=shape[0])

    def world_to_ndc(self, xyz_world, return_depth=False):
        """Nx3 world points -> Nx3 NDC (and N linear depths)."""
        xyzw = utils.hom(np.atleast_2d(xyz_world), 1.)
        if return_depth:
            cam = xyzw @ np.asarray(self.view_matrix).T
            depth = -cam[:, -2].copy()
            clip = cam @ np.asarray(self.proj_matrix).T
            return utils.dehom(clip), depth
        m = np.asarray(self.proj_matrix @ self.view_matrix)
        return utils.dehom(xyzw @ m.T)

    def ndc_to_pixel(self, ndc, origin='upper-left'):
        """NDC -> pixel coordinates, origin 'upper-left' (OpenCV) or 'lower-left' (OpenGL)."""
        assert origin in ['upper-left', 'lower-left']
        h, w = self.shape
        xy = (np.atleast_2d(ndc)[:, :2] + 1) * 0.5
        if origin == 'upper-left':
            xy[:, 1] = 1. - xy[:, 1]
        return xy * np.array([[w, h]])

    def object_to_pixel(self, *objs, return_depth=False):
        """Pixel coordinates (and depths) of every vertex of ``objs``."""
        if return_depth:
            ndc, z = self.world_to_ndc(utils.world_coordinates(*objs), return_depth=True)
            return self.ndc_to_pixel(ndc), z
        return self.ndc_to_pixel(self.world_to_ndc(utils.world_coordinates(*objs)))

    def bbox_object_to_pixel(self, *objs, return_depth=False):
        """Pixel coordinates (and depths) of the bounding-box corners of ``objs``."""
        if return_depth:
            ndc, z = self.world_to_ndc(utils.bbox_world_coordinates(*objs), return_depth=True)
            return self.ndc_to_pixel(ndc), z
        return self.ndc_to_pixel(self.world_to_ndc(utils.bbox_world_coordinates(*objs)))

    def look_at(self, look_at=None, look_from=None):
        """Point the camera's -Z axis at ``look_at`` (default origin), +Y up."""
        if look_from is None:
            look_from = self.bpy_camera.location
        if look_at is None:
            look_at = Vector([0, 0, 0])
        direction = Vector(look_at) - Vector(look_from)
        self.bpy_camera.rotation_euler = direction.to_track_quat('-Z', 'Y').to_euler()
        self.bpy_camera.location = Vector(look_from)
        self.update_view_matrix()
