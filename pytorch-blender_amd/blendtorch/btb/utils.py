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
    areas = [a for a in bpy.context.screen.areas if a.type == 'VIEW_3D']
    assert len(areas) > 0
    area = areas[0]
    region = max((r for r in area.regions if r.type == 'WINDOW'), key=lambda r: r.width)
    spaces = [s for s in area.spaces if s.type == 'VIEW_3D']
    assert len(spaces) > 0
    return area, spaces[0], region


def _eval(obj, depsgraph):
    return obj.evaluated_get(depsgraph or bpy.context.evaluated_depsgraph_get())


def object_coordinates(*objs, depsgraph=None):
    """Nx3 local vertex coordinates of the evaluated objects."""
    xyz = [np.asarray(v.co) for o in objs for v in _eval(o, depsgraph).data.vertices]
    return np.stack(xyz)


def world_coordinates(*objs, depsgraph=None):
    """Nx3 world vertex coordinates (``matrix_world @ v.co``)."""
    out = []
    for o in objs:
        e = _eval(o, depsgraph)
        out.extend(np.asarray(e.matrix_world @ v.co) for v in e.data.vertices)
    return np.stack(out)


def bbox_world_coordinates(*objs, depsgraph=None):
    """8*len(objs) x 3 world coordinates of the objects' bounding boxes."""
    out = []
    for o in objs:
        e = _eval(o, depsgraph)
        out.extend(np.asarray(e.matrix_world @ Vector(c)) for c in e.bound_box)
    return np.stack(out)


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
    """Fraction of N random vertices of ``obj`` whose ray from the camera hits ``obj`` first."""
    scene = scene or bpy.context.scene
    vl = view_layer or bpy.context.view_layer
    src = cam.bpy_camera.matrix_world.translation
    dist = dist or 1.70141e+38
    caminv = cam.bpy_camera.matrix_world.inverted()
    vis = 0
    for idx in np.random.choice(len(obj.data.vertices), size=N):
        dst_world = obj.matrix_world @ obj.data.vertices[idx].co
        d = (dst_world - src).normalized()
        dst_cam = caminv @ dst_world
        if dst_cam.z <= 0. and np.isfinite(np.asarray(d)).all():
            res, _, _, _, hit, _ = scene.ray_cast(vl, src, d, distance=dist)
            if res and hit == obj:
                vis += 1
    return vis / N


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
