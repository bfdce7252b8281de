"""Minimal numpy-backed ``mathutils`` (Vector, Matrix, Euler, Quaternion).

Only what blendtorch's Blender-side code and its test scenes use: 3/4-vectors
with attribute access and arithmetic, 3x3/4x4 matrices with ``@``,
``inverted``, ``normalized``, ``translation``, XYZ Euler angles and
``Vector.to_track_quat``.  Conventions follow Blender (column vectors,
``Matrix @ Vector``, Euler XYZ = Rz @ Ry @ Rx).
"""
import math

import numpy as np


class Vector:
    __slots__ = ('_v',)

    def __init__(self, seq=(0.0, 0.0, 0.0)):
        object.__setattr__(self, '_v', np.array(seq, dtype=np.float64).reshape(-1))

    # attribute access
    def __getattr__(self, name):
        idx = 'xyzw'.find(name)
        if len(name) == 1 and 0 <= idx < len(self._v):
            return float(self._v[idx])
        raise AttributeError(name)

    def __setattr__(self, name, value):
        idx = 'xyzw'.find(name)
        if len(name) == 1 and 0 <= idx < len(self._v):
            self._v[idx] = value
        else:
            raise AttributeError(name)

    def __len__(self):
        return len(self._v)

    def __getitem__(self, i):
        r = self._v[i]
        return Vector(r) if isinstance(i, slice) else float(r)

    def __setitem__(self, i, v):
        self._v[i] = v

    def __iter__(self):
        return iter(float(x) for x in self._v)

    def __array__(self, dtype=None, copy=None):
        return self._v.astype(dtype) if dtype is not None else self._v.copy()

    def __repr__(self):
        return f'Vector({tuple(round(float(x), 4) for x in self._v)})'

    def __eq__(self, o):
        return np.array_equal(self._v, np.asarray(o, dtype=np.float64))

    def __add__(self, o):
        return Vector(self._v + np.asarray(o, dtype=np.float64))

    __radd__ = __add__

    def __sub__(self, o):
        return Vector(self._v - np.asarray(o, dtype=np.float64))

    def __rsub__(self, o):
        return Vector(np.asarray(o, dtype=np.float64) - self._v)

    def __mul__(self, s):
        return Vector(self._v * s)

    __rmul__ = __mul__

    def __truediv__(self, s):
        return Vector(self._v / s)

    def __neg__(self):
        return Vector(-self._v)

    def __matmul__(self, o):
        if isinstance(o, Vector):
            return float(self._v @ o._v)
        return Vector(self._v @ np.asarray(o))

    def copy(self):
        return Vector(self._v)

    @property
    def length(self):
        return float(np.linalg.norm(self._v))

    def normalized(self):
        n = np.linalg.norm(self._v)
        return Vector(self._v / n if n > 0 else self._v)

    def normalize(self):
        n = np.linalg.norm(self._v)
        if n > 0:
            self._v /= n

    def dot(self, o):
        return float(self._v @ np.asarray(o, dtype=np.float64))

    def cross(self, o):
        return Vector(np.cross(self._v[:3], np.asarray(o, dtype=np.float64)[:3]))

    def to_4d(self):
        return Vector(list(self._v[:3]) + [1.0])

    def to_3d(self):
        return Vector(self._v[:3])

    def to_track_quat(self, track='-Z', up='Y'):
        """Rotation that points local axis ``track`` along this vector with the
        local ``up`` axis as close to world +Z as possible (Blender's rule for
        cameras: ``to_track_quat('-Z', 'Y')``)."""
        assert track == '-Z' and up == 'Y', 'only the camera convention is supported'
        d = self.normalized()._v[:3]
        z = -d
        world_up = np.array([0.0, 0.0, 1.0])
        x = np.cross(world_up, z)
        if np.linalg.norm(x) < 1e-9:
            x = np.array([1.0, 0.0, 0.0])
        x /= np.linalg.norm(x)
        y = np.cross(z, x)
        return Quaternion.from_matrix(np.stack([x, y, z], axis=1))


class Euler:
    __slots__ = ('_v', 'order')

    def __init__(self, angles=(0.0, 0.0, 0.0), order='XYZ'):
        object.__setattr__(self, '_v', np.array(angles, dtype=np.float64).reshape(3))
        object.__setattr__(self, 'order', order)

    def __getattr__(self, name):
        idx = 'xyz'.find(name)
        if len(name) == 1 and idx >= 0:
            return float(self._v[idx])
        raise AttributeError(name)

    def __setattr__(self, name, value):
        idx = 'xyz'.find(name)
        if len(name) == 1 and idx >= 0:
            self._v[idx] = value
        else:
            raise AttributeError(name)

    def __getitem__(self, i):
        return float(self._v[i])

    def __setitem__(self, i, v):
        self._v[i] = v

    def __len__(self):
        return 3

    def __iter__(self):
        return iter(float(x) for x in self._v)

    def __array__(self, dtype=None, copy=None):
        return self._v.astype(dtype) if dtype is not None else self._v.copy()

    def __repr__(self):
        return f'Euler({tuple(round(float(x), 4) for x in self._v)})'

    def to_matrix(self):
        rx, ry, rz = self._v
        cx, sx, cy, sy, cz, sz = math.cos(rx), math.sin(rx), math.cos(ry), math.sin(ry), math.cos(rz), math.sin(rz)
        Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
        Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
        Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
        return Matrix(Rz @ Ry @ Rx)


def _euler_from_rot(R):
    R = np.asarray(R, dtype=np.float64)[:3, :3]
    sy = -R[2, 0]
    sy = max(-1.0, min(1.0, sy))
    ry = math.asin(sy)
    if abs(math.cos(ry)) > 1e-9:
        rx = math.atan2(R[2, 1], R[2, 2])
        rz = math.atan2(R[1, 0], R[0, 0])
    else:  # gimbal lock
        rx = math.atan2(-R[1, 2], R[1, 1])
        rz = 0.0
    return Euler((rx, ry, rz))


class Quaternion:
    def __init__(self, wxyz=(1.0, 0.0, 0.0, 0.0)):
        self._q = np.array(wxyz, dtype=np.float64)

    @staticmethod
    def from_matrix(R):
        R = np.asarray(R, dtype=np.float64)
        t = np.trace(R)
        if t > 0:
            s = math.sqrt(t + 1.0) * 2
            w, x, y, z = 0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s
        elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
            s = math.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
            w, x, y, z = (R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s
        elif R[1, 1] > R[2, 2]:
            s = math.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
            w, x, y, z = (R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s
        else:
            s = math.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
            w, x, y, z = (R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s
        return Quaternion((w, x, y, z))

    def to_matrix(self):
        w, x, y, z = self._q / np.linalg.norm(self._q)
        return Matrix(np.array([
            [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
            [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
            [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]]))

    def to_euler(self, order='XYZ'):
        return _euler_from_rot(self.to_matrix())


class Matrix:
    def __init__(self, rows=None):
        if rows is None:
            rows = np.eye(4)
        self._m = np.array(rows, dtype=np.float64)

    @staticmethod
    def Identity(n):
        return Matrix(np.eye(n))

    @staticmethod
    def Translation(v):
        m = np.eye(4)
        m[:3, 3] = np.asarray(v, dtype=np.float64)[:3]
        return Matrix(m)

    def __array__(self, dtype=None, copy=None):
        return self._m.astype(dtype) if dtype is not None else self._m.copy()

    def __getitem__(self, i):
        r = self._m[i]
        return Vector(r) if r.ndim == 1 else r

    def __len__(self):
        return len(self._m)

    def __repr__(self):
        return f'Matrix({np.round(self._m, 4).tolist()})'

    def __eq__(self, o):
        return np.allclose(self._m, np.asarray(o))

    def __matmul__(self, o):
        if isinstance(o, Matrix):
            return Matrix(self._m @ o._m)
        v = np.asarray(o, dtype=np.float64)
        n = self._m.shape[0]
        if n == 4 and v.shape[0] == 3:   # Blender: 4x4 @ Vector3 applies w=1
            r = self._m @ np.append(v, 1.0)
            return Vector(r[:3] / r[3] if r[3] not in (0.0, 1.0) else r[:3])
        return Vector(self._m @ v)

    def inverted(self):
        return Matrix(np.linalg.inv(self._m))

    def transposed(self):
        return Matrix(self._m.T)

    def normalized(self):
        m = self._m.copy()
        k = min(3, m.shape[0])
        for c in range(k):
            n = np.linalg.norm(m[:k, c])
            if n > 0:
                m[:k, c] /= n
        return Matrix(m)

    def copy(self):
        return Matrix(self._m)

    @property
    def translation(self):
        return Vector(self._m[:3, 3])

    @translation.setter
    def translation(self, v):
        self._m[:3, 3] = np.asarray(v, dtype=np.float64)[:3]

    def to_3x3(self):
        return Matrix(self._m[:3, :3])

    def to_4x4(self):
        m = np.eye(4)
        m[:3, :3] = self._m[:3, :3]
        if self._m.shape[0] == 4:
            m = self._m.copy()
        return Matrix(m)

    def to_euler(self, order='XYZ'):
        return _euler_from_rot(self.normalized()._m)

    def to_scale(self):
        return Vector(np.linalg.norm(self._m[:3, :3], axis=0))

    def decompose(self):
        loc = Vector(self._m[:3, 3])
        scale = self.to_scale()
        rot = Quaternion.from_matrix(self.normalized()._m[:3, :3])
        return loc, rot, scale
