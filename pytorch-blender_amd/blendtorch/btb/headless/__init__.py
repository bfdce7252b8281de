"""Headless Blender stand-in: a pure-Python ``bpy`` subset + a ``blender`` CLI.

Blender is not part of this stack, yet ``blendtorch.btb`` is Blender-side
code.  This package emulates the slice of Blender that btb and typical
producer scripts touch, so the Blender-side API runs -- and is tested --
exactly as it would inside Blender:

* ``bpy``: ``context`` (scene, view_layer, screen with a VIEW_3D area,
  space_data, evaluated_depsgraph_get), ``data`` (objects, collections,
  materials, meshes), ``app`` (background, handlers.frame_change_pre/post,
  version), ``types.SpaceView3D.draw_handler_add/remove``,
  ``ops.screen.animation_play/animation_cancel``; ``Scene.frame_set`` runs
  the frame-change handlers like Blender (frame_current already updated
  in pre handlers); ``Object.matrix_world``/``calc_matrix_camera`` follow
  Blender's conventions (camera looks down -Z, sensor_fit AUTO).
* ``mathutils``: see :mod:`.mathutils`.
* ``gpu``/``bgl``: ``GPUOffScreen.draw_view3d`` rasterises the scene's mesh
  objects (as oriented boxes) with the native renderer; the image is read
  back with ``offscreen.texture_color.read()``.
* ``blender`` CLI (:func:`main`): ``blender [scene] [--background]
  [--python-use-system-env] [--python-exit-code N] --python script -- args``
  and ``--version``.  In UI mode (no ``--background``) it runs a frame loop
  that drives ``animation_play`` and POST_PIXEL draw handlers, like
  Blender's timer-driven playback.

Scenes: a ``.blend`` path selects a built-in preset by file stem
(``cube``, ``falling_cubes``, ``cam``, ``supershape``, ``cartpole``);
anything else gives Blender's default startup scene (Cube, Camera, Light).
"""
from __future__ import annotations

import math
import sys
import time
import types
from pathlib import Path

import numpy as np

from . import mathutils as mu
from .mathutils import Euler, Matrix, Vector, _euler_from_rot

# ---------------------------------------------------------------------------
# data model
# ---------------------------------------------------------------------------
_CUBE_VERTS = [(1, 1, 1), (1, 1, -1), (1, -1, 1), (1, -1, -1), (-1, 1, 1), (-1, 1, -1), (-1, -1, 1), (-1, -1, -1)]


class MeshVertex:
    def __init__(self, co, index):
        self.co = Vector(co)
        self.index = index


class Mesh:
    def __init__(self, name, verts=_CUBE_VERTS):
        self.name = name
        self.vertices = [MeshVertex(v, i) for i, v in enumerate(verts)]
        self.materials = []
        self.users = 1


class CameraData:
    def __init__(self, name, type='PERSP', lens=50.0, sensor_width=36.0, sensor_height=24.0, ortho_scale=7.314,
                 clip_start=0.1, clip_end=100.0):
        self.name = name
        self.type = type
        self.lens = lens
        self.sensor_width = sensor_width
        self.sensor_height = sensor_height
        self.sensor_fit = 'AUTO'
        self.ortho_scale = ortho_scale
        self.clip_start = clip_start
        self.clip_end = clip_end
        self.shift_x = 0.0
        self.shift_y = 0.0


class LightData:
    def __init__(self, name, type='POINT', energy=1000.0):
        self.name = name
        self.type = type
        self.energy = energy


class Material:
    def __init__(self, name):
        self.name = name
        self.diffuse_color = (0.8, 0.8, 0.8, 1.0)
        self.users = 1


class Object:
    def __init__(self, name, data=None, type='MESH', location=(0, 0, 0), rotation=(0, 0, 0), scale=(1, 1, 1)):
        self.name = name
        self.data = data
        self.type = type
        self.location = Vector(location)
        self.rotation_euler = Euler(rotation)
        self.scale = Vector(scale)
        self.parent = None
        self.users = 1
        self.active_material = None
        self.hide_render = False
        self.rigid_body = None

    def __repr__(self):
        return f'<headless Object {self.name!r} ({self.type})>'

    # Blender accepts any 3-sequence for these; keep them as mathutils types
    @property
    def location(self):
        return self._location

    @location.setter
    def location(self, v):
        self._location = v if isinstance(v, Vector) else Vector(v)

    @property
    def rotation_euler(self):
        return self._rotation

    @rotation_euler.setter
    def rotation_euler(self, v):
        self._rotation = v if isinstance(v, Euler) else Euler(v)

    @property
    def scale(self):
        return self._scale

    @scale.setter
    def scale(self, v):
        self._scale = v if isinstance(v, Vector) else Vector(v)

    @property
    def matrix_world(self):
        m = np.eye(4)
        m[:3, :3] = np.asarray(self.rotation_euler.to_matrix()) @ np.diag(np.asarray(self.scale))
        m[:3, 3] = np.asarray(self.location)
        mw = Matrix(m)
        if self.parent is not None:
            mw = self.parent.matrix_world @ mw
        return mw

    @matrix_world.setter
    def matrix_world(self, M):
        M = Matrix(np.asarray(M))
        self.location = Vector(np.asarray(M)[:3, 3])
        self.scale = M.to_scale()
        self.rotation_euler = M.to_euler()

    def evaluated_get(self, depsgraph):
        return self

    @property
    def bound_box(self):
        v = np.array([np.asarray(x.co) for x in self.data.vertices])
        lo, hi = v.min(0), v.max(0)
        # Blender's bound_box corner order
        return [(lo[0], lo[1], lo[2]), (lo[0], lo[1], hi[2]), (lo[0], hi[1], hi[2]), (lo[0], hi[1], lo[2]),
                (hi[0], lo[1], lo[2]), (hi[0], lo[1], hi[2]), (hi[0], hi[1], hi[2]), (hi[0], hi[1], lo[2])]

    def calc_matrix_camera(self, depsgraph, x=None, y=None, scale_x=1.0, scale_y=1.0):
        """OpenGL-style projection of a camera object (Blender semantics,
        sensor_fit AUTO: the larger image side spans the sensor width)."""
        cam = self.data
        scene = _state.scene
        if x is None:
            x = scene.render.resolution_x * scene.render.resolution_percentage / 100.0
        if y is None:
            y = scene.render.resolution_y * scene.render.resolution_percentage / 100.0
        x, y = float(x) * scale_x, float(y) * scale_y
        n, f = cam.clip_start, cam.clip_end
        P = np.zeros((4, 4))
        if cam.type == 'ORTHO':
            sx = 2.0 / cam.ortho_scale if x >= y else 2.0 / cam.ortho_scale * y / x
            sy = sx * x / y
            P[0, 0], P[1, 1] = sx, sy
            P[2, 2] = -2.0 / (f - n)
            P[2, 3] = -(f + n) / (f - n)
            P[3, 3] = 1.0
        else:
            sx = 2.0 * cam.lens / cam.sensor_width if x >= y else 2.0 * cam.lens / cam.sensor_width * y / x
            sy = sx * x / y
            P[0, 0], P[1, 1] = sx, sy
            P[2, 2] = -(f + n) / (f - n)
            P[2, 3] = -2.0 * f * n / (f - n)
            P[3, 2] = -1.0
        return Matrix(P)

    def to_mesh(self):
        return self.data


class _Collection(dict):
    """Name-indexed bpy_collection (iterates values like Blender)."""

    def __iter__(self):
        return iter(list(self.values()))

    def __getitem__(self, k):
        if isinstance(k, int):
            return list(self.values())[k]
        return dict.__getitem__(self, k)

    def new(self, name, data=None):
        if self is _state.data.materials:
            obj = Material(name)
        elif self is _state.data.meshes:
            obj = Mesh(name, verts=[])
        else:
            obj = Object(name, data)
        self[name] = obj
        return obj

    def remove(self, obj, do_unlink=True):
        self.pop(obj.name, None)

    @property
    def all_objects(self):
        return list(self.values())


class ObjCollection:
    def __init__(self, name, objects):
        self.name = name
        self.objects = _Collection((o.name, o) for o in objects)
        self.all_objects = list(objects)


class RenderSettings:
    def __init__(self, x=1920, y=1080, percentage=100, fps=24):
        self.resolution_x = x
        self.resolution_y = y
        self.resolution_percentage = percentage
        self.fps = fps
        self.fps_base = 1.0


class PointCache:
    def __init__(self, start=1, end=250):
        self.frame_start = start
        self.frame_end = end


class RigidBodyObject:
    """``Object.rigid_body``: an active body with a box collision shape."""

    def __init__(self, type='ACTIVE', collision_shape='BOX', mass=1.0):
        self.type = type
        self.collision_shape = collision_shape
        self.mass = mass


class RigidBodyWorld:
    """Scene rigid-body world.  Objects with a ``rigid_body`` (active, box
    collision shape) are simulated by the native solver (csrc/sim/physics.cpp):
    at the cache's first frame the world resets to the objects' current pose
    (the pose ``pre_animation`` handlers just set), every later frame advances
    it by one frame and writes the evaluated pose back -- between the
    frame_change_pre and frame_change_post handlers, as Blender's depsgraph
    evaluation does."""

    def __init__(self):
        self.point_cache = PointCache()
        self.enabled = True
        self._world = None
        self._objects = []

    def _bodies(self, scene):
        return [o for o in scene.objects if getattr(o, 'rigid_body', None) is not None and o.type == 'MESH']

    def evaluate(self, scene):
        if not self.enabled:
            return
        objs = self._bodies(scene)
        if not objs:
            return
        from ... import _native
        start = self.point_cache.frame_start
        if self._world is None or scene.frame_current <= start or objs != self._objects:
            self._world = _native.RigidWorld(float(scene.plane_z if scene.plane_z is not None else 0.0))
            self._objects = objs
            centers = np.array([np.asarray(o.location, dtype=np.float64) for o in objs])
            rots = np.array([np.asarray(o.rotation_euler.to_matrix(), dtype=np.float64) for o in objs])
            halves = np.array([np.asarray(o.scale, dtype=np.float64) for o in objs])   # unit cube * scale
            self._world.set_bodies(centers, rots, halves)
            return
        self._world.step(1.0 / max(1, scene.render.fps))
        for o, c, R in zip(objs, self._world.centers(), self._world.rotations()):
            o.location = Vector(c)
            o.rotation_euler = _euler_from_rot(np.asarray(R))


class Scene:
    def __init__(self, name='Scene'):
        self.name = name
        self.objects = _Collection()
        self.camera = None
        self.frame_start = 1
        self.frame_end = 250
        self.frame_current = 1
        self.render = RenderSettings()
        self.rigidbody_world = None
        self.light_power = 1000.0
        self.plane_z = None

    def frame_set(self, frame, subframe=0.0):
        """Jump to ``frame``: frame_current is updated, then the pre handlers,
        the (trivial) depsgraph evaluation and the post handlers run."""
        self.frame_current = int(frame)
        for h in list(_state.app.handlers.frame_change_pre):
            h(self, _state.depsgraph)
        if self.rigidbody_world is not None:
            self.rigidbody_world.evaluate(self)
        for h in list(_state.app.handlers.frame_change_post):
            h(self, _state.depsgraph)

    def ray_cast(self, view_layer, origin, direction, distance=1.70141e+38):
        """Nearest hit of a ray with the mesh objects (treated as oriented boxes)."""
        o = np.asarray(origin, dtype=np.float64)[:3]
        d = np.asarray(direction, dtype=np.float64)[:3]
        best = (False, Vector((0, 0, 0)), Vector((0, 0, 0)), -1, None, Matrix())
        tbest = distance
        for obj in self.objects:
            if obj.type != 'MESH':
                continue
            M = np.asarray(obj.matrix_world)
            Minv = np.linalg.inv(M)
            lo = Minv[:3, :3] @ o + Minv[:3, 3]
            ld = Minv[:3, :3] @ d
            v = np.array([np.asarray(x.co) for x in obj.data.vertices]) if obj.data.vertices else np.zeros((1, 3))
            bmin, bmax = v.min(0), v.max(0)
            t0, t1 = 0.0, tbest
            hit = True
            for a in range(3):
                if abs(ld[a]) < 1e-12:
                    if lo[a] < bmin[a] or lo[a] > bmax[a]:
                        hit = False
                        break
                    continue
                ta, tb = (bmin[a] - lo[a]) / ld[a], (bmax[a] - lo[a]) / ld[a]
                t0, t1 = max(t0, min(ta, tb)), min(t1, max(ta, tb))
                if t0 > t1:
                    hit = False
                    break
            if hit and t0 < tbest:
                tbest = t0
                p = o + t0 * d
                best = (True, Vector(p), Vector((0, 0, 1)), 0, obj, Matrix(M))
        return best


class Depsgraph:
    def update(self):
        pass


class _Shading:
    def __init__(self):
        self.type = 'SOLID'


class _Overlay:
    def __init__(self):
        self.show_overlays = True


class SpaceView3D:
    _draw_handlers = []

    def __init__(self):
        self.type = 'VIEW_3D'
        self.shading = _Shading()
        self.overlay = _Overlay()

    @classmethod
    def draw_handler_add(cls, fn, args, region_type, draw_type):
        h = (fn, tuple(args), region_type, draw_type)
        cls._draw_handlers.append(h)
        return h

    @classmethod
    def draw_handler_remove(cls, handle, region_type):
        if handle in cls._draw_handlers:
            cls._draw_handlers.remove(handle)


class Region:
    def __init__(self, type='WINDOW', width=1280, height=720):
        self.type = type
        self.width = width
        self.height = height


class Area:
    def __init__(self):
        self.type = 'VIEW_3D'
        self.spaces = [SpaceView3D()]
        self.regions = [Region('HEADER', 1280, 26), Region('WINDOW', 1280, 720)]


class Screen:
    def __init__(self):
        self.areas = [Area()]


# ---------------------------------------------------------------------------
# module state + scene presets
# ---------------------------------------------------------------------------
class _State:
    pass


_state = _State()


def _default_objects(scene):
    cube = Object('Cube', Mesh('Cube'), 'MESH')
    cam = Object('Camera', CameraData('Camera'), 'CAMERA', location=(7.358891, -6.925791, 4.958309),
                 rotation=(1.109319, 0.0, 0.814928))
    light = Object('Light', LightData('Light'), 'LIGHT', location=(4.076245, 1.005454, 5.903862))
    for o in (cube, cam, light):
        scene.objects[o.name] = o
    scene.camera = cam
    return cube, cam, light


def make_scene(path=None):
    """Build the scene for a ``.blend`` path (preset by file stem)."""
    stem = Path(str(path)).stem if path else ''
    sc = Scene()
    cube, cam, light = _default_objects(sc)
    if stem == 'cube':
        sc.render = RenderSettings(640, 480, 100, 60)
        sc.plane_z = -2.0
    elif stem == 'falling_cubes':
        sc.render = RenderSettings(640, 480, 100, 60)
        sc.objects.pop('Cube')
        cubes = []
        for i in range(7):
            c = Object(f'Cube.{i:03d}', Mesh(f'Cube.{i:03d}'), 'MESH', location=(0, 0, 2 * i))
            c.rigid_body = RigidBodyObject()
            sc.objects[c.name] = c
            cubes.append(c)
        _state.collections['Cubes'] = ObjCollection('Cubes', cubes)
        cam.location = Vector((14.5, -15.712, 16.754))
        sc.plane_z = -2.0
        sc.rigidbody_world = RigidBodyWorld()
    elif stem == 'cam':
        sc.render = RenderSettings(640, 480, 100, 24)
        sc.objects.pop('Camera')
        ortho = Object('CamOrtho', CameraData('CamOrtho', 'ORTHO', ortho_scale=4.0, clip_start=1.0, clip_end=10.0),
                       'CAMERA', location=(0, 0, 7))
        proj = Object('CamProj', CameraData('CamProj', 'PERSP', lens=50.0, clip_start=1.0, clip_end=10.0),
                      'CAMERA', location=(0, 0, 7))
        sc.objects[ortho.name] = ortho
        sc.objects[proj.name] = proj
        sc.camera = proj
    elif stem == 'supershape':
        sc.render = RenderSettings(64, 64, 100, 200)
        cam.data.lens = 150.0
    elif stem == 'cartpole':
        sc.render = RenderSettings(1920, 1080, 25, 60)
        sc.rigidbody_world = RigidBodyWorld()
    return sc


def reset(scene_path=None, background=True):
    """(Re)initialise the emulated Blender session."""
    _state.collections = _Collection()
    _state.depsgraph = Depsgraph()
    app = types.SimpleNamespace(
        background=background,
        version=(2, 90, 0),
        version_string='2.90.0 (headless)',
        binary_path=sys.argv[0],
        handlers=types.SimpleNamespace(frame_change_pre=[], frame_change_post=[], render_pre=[], render_post=[],
                                       load_post=[]),
    )
    _state.app = app
    _state.scene = make_scene(scene_path)
    _state.screen = Screen()
    _state.playing = False
    SpaceView3D._draw_handlers = []
    _state.data = types.SimpleNamespace(
        objects=_state.scene.objects, collections=_state.collections, materials=_Collection(),
        meshes=_Collection(), cameras=_Collection(), lights=_Collection(), scenes=_Collection(Scene=_state.scene))
    _state.context = types.SimpleNamespace(
        scene=_state.scene, view_layer=types.SimpleNamespace(name='ViewLayer'), screen=_state.screen,
        space_data=None, window_manager=types.SimpleNamespace(), evaluated_depsgraph_get=lambda: _state.depsgraph)
    return _state


# ---------------------------------------------------------------------------
# bpy / gpu / bgl module objects
# ---------------------------------------------------------------------------
def _animation_play(*args, **kwargs):
    if not _state.app.background:
        _state.playing = True
    return {'FINISHED'}


def _animation_cancel(restore_frame=True):
    _state.playing = False
    return {'FINISHED'}


class _Texture:
    def __init__(self, off):
        self._off = off

    def read(self):
        return self._off._buffer


class GPUOffScreen:
    """Offscreen target; ``draw_view3d`` renders with the native rasteriser.

    Pixels are stored bottom-up (OpenGL readback order) in RGBA u8.
    """

    def __init__(self, width, height):
        self.width, self.height = int(width), int(height)
        self._buffer = np.zeros((self.height, self.width, 4), np.uint8)
        self.color_texture = 1
        self.texture_color = _Texture(self)

    def bind(self):
        import contextlib
        return contextlib.nullcontext(self)

    def free(self):
        pass

    def draw_view3d(self, scene, view_layer, space, region, view_matrix, proj_matrix, do_color_management=False):
        from ... import _native
        V = np.asarray(view_matrix, dtype=np.float64)
        P = np.asarray(proj_matrix, dtype=np.float64)
        if abs(P[3, 3]) > 0.5:
            raise NotImplementedError('headless renderer supports perspective cameras only')
        C = np.linalg.inv(V)                    # camera-to-world
        rot = C[:3, :3] / np.linalg.norm(C[:3, :3], axis=0)
        # P[0,0] = 2 f / W  ->  lens/sensor = P00 / 2 for the wide side
        W, H = self.width, self.height
        fx = P[0, 0] * W / 2.0
        lens, sensor = fx, float(max(W, H))
        light = next((o for o in scene.objects if o.type == 'LIGHT'), None)
        lloc = list(np.asarray(light.location)) if light is not None else [4.0, 1.0, 6.0]
        boxes = []
        for o in scene.objects:
            if o.type != 'MESH' or o.hide_render or not o.data.vertices:
                continue
            M = np.asarray(o.matrix_world)
            v = np.array([np.asarray(x.co) for x in o.data.vertices])
            lo, hi = v.min(0), v.max(0)
            ctr_local = (lo + hi) / 2
            half = (hi - lo) / 2 * np.linalg.norm(M[:3, :3], axis=0)
            R = M[:3, :3] / np.maximum(np.linalg.norm(M[:3, :3], axis=0), 1e-12)
            ctr = M[:3, :3] @ ctr_local + M[:3, 3]
            mat = o.active_material or (o.data.materials[0] if o.data.materials else None)
            col = tuple(mat.diffuse_color[:3]) if mat is not None else (0.8, 0.8, 0.8)
            boxes.append((list(ctr), list(half), list(R.reshape(-1)), list(col)))
        pz = scene.plane_z if scene.plane_z is not None else -1e9
        img = _native.render_boxes(W, H, 4, True, list(C[:3, 3]), list(rot.reshape(-1)), lens, sensor, lloc,
                                   getattr(light.data, 'energy', 1000.0) if light is not None else 1000.0, pz,
                                   10.0 if scene.plane_z is not None else 0.0, boxes)
        self._buffer[...] = img


def _make_modules():
    bpy = types.ModuleType('bpy')
    bpy.__headless__ = True
    bpy.app = _state.app
    bpy.context = _state.context
    bpy.data = _state.data
    bpy.types = types.SimpleNamespace(SpaceView3D=SpaceView3D, Object=Object, Scene=Scene, Mesh=Mesh,
                                      Camera=CameraData, Collection=_Collection, Material=Material)
    bpy.ops = types.SimpleNamespace(screen=types.SimpleNamespace(animation_play=_animation_play,
                                                                 animation_cancel=_animation_cancel))
    bpy.utils = types.SimpleNamespace(register_class=lambda c: None, unregister_class=lambda c: None)
    mathutils = types.ModuleType('mathutils')
    for n in ('Vector', 'Matrix', 'Euler', 'Quaternion'):
        setattr(mathutils, n, getattr(mu, n))
    gpu = types.ModuleType('gpu')
    gpu.types = types.SimpleNamespace(GPUOffScreen=GPUOffScreen)
    bgl = types.ModuleType('bgl')
    for k, v in dict(GL_TEXTURE0=0x84C0, GL_TEXTURE_2D=0x0DE1, GL_RGBA=0x1908, GL_RGB=0x1907,
                     GL_UNSIGNED_BYTE=0x1401).items():
        setattr(bgl, k, v)
    bgl.glActiveTexture = lambda *a: None
    bgl.glBindTexture = lambda *a: None
    bmesh = types.ModuleType('bmesh')
    bpy_extras = types.ModuleType('bpy_extras')
    return {'bpy': bpy, 'mathutils': mathutils, 'gpu': gpu, 'bgl': bgl, 'bmesh': bmesh, 'bpy_extras': bpy_extras}


_modules = None


def install(scene_path=None, background=True):
    """Install the emulated modules into ``sys.modules`` (fresh session).

    The module objects are created once and re-pointed at the new session
    state on later calls, so code that already did ``import bpy`` sees the
    new scene.
    """
    global _modules
    reset(scene_path, background)
    if _modules is None:
        _modules = _make_modules()
    else:
        bpy = _modules['bpy']
        bpy.app, bpy.context, bpy.data = _state.app, _state.context, _state.data
    sys.modules.update(_modules)
    return _modules['bpy']


def is_headless():
    b = sys.modules.get('bpy')
    return b is not None and getattr(b, '__headless__', False)


def run_event_loop(max_idle_s=None):
    """UI-mode main loop: while an animation plays, step frames at the scene
    fps-agnostic maximum rate and run POST_PIXEL draw handlers after each frame
    (twice, as Blender may redraw a frame more than once)."""
    space = _state.screen.areas[0].spaces[0]
    idle_since = time.time()
    def redraw():
        for _ in range(2):
            for fn, args, region, kind in list(SpaceView3D._draw_handlers):
                _state.context.space_data = space
                try:
                    fn(*args)
                finally:
                    _state.context.space_data = None

    while True:
        if _state.playing:
            # the viewport shows the current frame before the timer advances
            redraw()
            if not _state.playing:
                continue
            sc = _state.scene
            nxt = sc.frame_current + 1
            if nxt > sc.frame_end:
                nxt = sc.frame_start
            sc.frame_set(nxt)
            idle_since = time.time()
        else:
            if max_idle_s is not None and time.time() - idle_since > max_idle_s:
                return
            time.sleep(0.01)


def main(argv=None):
    """``blender`` command-line stand-in."""
    import runpy
    argv = list(sys.argv[1:] if argv is None else argv)
    if '--version' in argv or '-v' in argv:
        print('Blender 2.90.0 (blendtorch headless)')
        print('\tbuild: headless emulation')
        return 0
    script_args = []
    if '--' in argv:
        i = argv.index('--')
        argv, script_args = argv[:i], argv[i:]
    background = False
    exit_code = 0
    scripts = []
    scene = None
    it = iter(range(len(argv)))
    i = 0
    while i < len(argv):
        a = argv[i]
        if a in ('-b', '--background'):
            background = True
        elif a == '--python-use-system-env':
            pass
        elif a == '--python-exit-code':
            exit_code = int(argv[i + 1])
            i += 1
        elif a in ('-P', '--python'):
            scripts.append(argv[i + 1])
            i += 1
        elif not a.startswith('-') and scene is None:
            scene = a
        i += 1
    install(scene, background)
    sys.argv = ['blender'] + argv + script_args
    for s in scripts:
        try:
            runpy.run_path(s, run_name='__main__')
        except SystemExit as e:
            if e.code not in (None, 0):
                return e.code if isinstance(e.code, int) else 1
        except Exception:
            import traceback
            traceback.print_exc()
            if exit_code:
                return exit_code
            if background:
                return 1
    if background:
        return 0
    import os
    idle = os.environ.get('BLENDTORCH_HEADLESS_IDLE_EXIT')
    run_event_loop(max_idle_s=float(idle) if idle else None)
    return 0
