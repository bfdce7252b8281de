"""Scene helpers (reference: pkg_blender/blendtorch/btb/utils.py).

``find_first_view3d`` returns ``(area, space, region)`` of the first 3D view
(the reference docstring lists another order; the code -- and this module --
return area, space, region).  Coordinate helpers stack vertex positions of
evaluated objects; ``hom``/``dehom`` convert to/from homogeneous coordinates.
"""
import bpy
import numpy as np
from mathutils import Vector


def find_first_view3d():
    """``(area, space, region)`` of the first VIEW_3D area (widest WINDOW region)."""
    area = next((a for a in bpy.context.screen.areas if a.type == 'VIEW_3D'), None)
    assert area is not None, 'no 3D view in the current screen'
    space = next((s for s in area.spaces if s.type == 'VIEW_3D'), None)
    assert space is not None, 'the 3D view area has no VIEW_3D space'
    windows = [r for r in area.regions if r.type == 'WINDOW']
    return area, space, max(windows, key=lambda r: r.width)


def _rows(objs, depsgraph, points):
    """Stack ``points(evaluated_object)`` (an iterable of 3-vectors) over
    ``objs``, evaluated after modifiers in ``depsgraph`` (default: the
    context's)."""
    dg = depsgraph or bpy.context.evaluated_depsgraph_get()
    return np.stack([np.asarray(p) for o in objs for p in points(o.evaluated_get(dg))])


def object_coordinates(*objs, depsgraph=None):
    """Nx3 local vertex coordinates of the evaluated objects."""
    return _rows(objs, depsgraph, lambda e: (v.co for v in e.data.vertices))


def world_coordinates(*objs, depsgraph=None):
    """Nx3 world vertex coordinates (``matrix_world @ v.co``)."""
    return _rows(objs, depsgraph, lambda e: (e.matrix_world @ v.co for v in e.data.vertices))


def bbox_world_coordinates(*objs, depsgraph=None):
    """8*len(objs) x 3 world coordinates of the objects' bounding boxes."""
    return _rows(objs, depsgraph, lambda e: (e.matrix_world @ Vector(c) for c in e.bound_box))


def hom(x, v=1.):
    """Append a homogeneous coordinate ``v`` to every row of ``x``."""
    return np.concatenate((x, np.full((x.shape[0], 1), v, dtype=x.dtype)), -1)


def dehom(x):
    """Divide by and drop the last coordinate."""
    return x[..., :-1] / x[..., -1:]


def random_spherical_loc(radius_range=None, theta_range=None, phi_range=None):
    """Random point on a spherical shell (not area-uniform), as in the reference."""
    radius_range = radius_range or (1, 1)
    theta_range = theta_range or (0, np.pi)
    phi_range = phi_range or (0, 2 * np.pi)
    r = np.random.uniform(*radius_range)
    t = np.random.uniform(*theta_range)
    p = np.random.uniform(*phi_range)
    return np.array([np.sin(t) * np.cos(p), np.sin(t) * np.sin(p), np.cos(t)]) * r


def compute_object_visibility(obj, cam, N=25, scene=None, view_layer=None, dist=None):
    """Fraction of N random vertices of ``obj`` whose ray from the camera hits ``obj`` first.

    Monte-Carlo estimate: a sampled vertex counts when it lies in front of
    the camera (negative camera-space z) and the scene ray cast from the
    camera origin towards it reports ``obj`` as the first hit."""
    scene = scene or bpy.context.scene
    layer = view_layer or bpy.context.view_layer
    cam_world = cam.bpy_camera.matrix_world
    origin, to_cam = cam_world.translation, cam_world.inverted()
    max_dist = dist or 1.70141e+38

    def visible(vertex_index):
        target = obj.matrix_world @ obj.data.vertices[vertex_index].co
        if (to_cam @ target).z > 0.:
            return False                      # behind the camera
        ray = (target - origin).normalized()
        if not np.isfinite(np.asarray(ray)).all():
            return False
        hit, _loc, _normal, _face, first, _m = scene.ray_cast(layer, origin, ray, distance=max_dist)
        return bool(hit) and first == obj

    picks = np.random.choice(len(obj.data.vertices), size=N)
    return sum(visible(i) for i in picks) / N


def scene_stats():
    """``{collection_name: (n_active, n_orphaned)}`` over bpy.data collections."""
    stats = {}
    for attr in dir(bpy.data):
        coll = getattr(bpy.data, attr, None)
        objs = getattr(coll, 'all_objects', None)
        if objs is None:
            try:
                objs = list(coll.values())
            except (AttributeError, TypeError):
                continue
        if not objs:
            continue
        users = [getattr(o, 'users', 1) for o in objs]
        stats[attr] = (sum(u > 0 for u in users), sum(u == 0 for u in users))
    return stats
