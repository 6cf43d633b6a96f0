"""Host-side SE(3) value types, API-compatible with the reference's artelib subset.

The registration boundary returns ``HomogeneousMatrix`` (keyframe.py:259) and the callers compose
4x4 transforms with it (run_scanmatcher.py:221, loopclosing.py:167-200). This module provides the
same surface -- ``HomogeneousMatrix`` (artelib/homogeneousmatrix.py:16-144), ``Euler``,
``Quaternion``, ``RotationMatrix`` and the transform-list helpers (:147-212) -- with the same
conventions: Euler XYZ in mobile axes, R = Rx(a) Ry(b) Rz(g) (artelib/tools.py:226-238);
quaternions ordered [w, x, y, z] (tools.py:92-172); ``rot2euler`` returns both solutions and
clamps R[0, 2] IN PLACE (tools.py:241-275; HomogeneousMatrix.R() is a view), a quirk kept on
purpose because ``euler()`` may then touch ``.array`` of a near-singular pose.

Host-only: nothing here runs on the GPU.
"""
from __future__ import annotations

import numpy as np


# ------------------------------------------------------------------------------------------
# conversions
# ------------------------------------------------------------------------------------------
def _rx(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])


def _ry(b):
    c, s = np.cos(b), np.sin(b)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def _rz(g):
    c, s = np.cos(g), np.sin(g)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def euler2rot(abg):
    """XYZ mobile axes: R = Rx(alpha) @ Ry(beta) @ Rz(gamma)."""
    return np.matmul(np.matmul(_rx(abg[0]), _ry(abg[1])), _rz(abg[2]))


def quaternion2rot(q):
    w, x, y, z = q[0], q[1], q[2], q[3]
    R = np.eye(3)
    R[0, 0] = 1 - 2 * y ** 2 - 2 * z ** 2
    R[0, 1] = 2 * x * y - 2 * z * w
    R[0, 2] = 2 * x * z + 2 * y * w
    R[1, 0] = 2 * x * y + 2 * z * w
    R[1, 1] = 1 - 2 * x ** 2 - 2 * z ** 2
    R[1, 2] = 2 * y * z - 2 * x * w
    R[2, 0] = 2 * x * z - 2 * y * w
    R[2, 1] = 2 * y * z + 2 * x * w
    R[2, 2] = 1 - 2 * x ** 2 - 2 * y ** 2
    return R


def _sgn(v):
    return 1 if v >= 0 else -1


def rot2quaternion(R):
    """[w, x, y, z] from a rotation matrix (Sarabandi & Thomas closed form, trace clamped >= 0)."""
    R = R[0:3, 0:3]
    s = np.sqrt(max(0.0, np.trace(R) + 1)) / 2.0
    k = [R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]]
    dom = int(np.argmax(np.diag(R)))
    if dom == 0:
        k1 = [R[0, 0] - R[1, 1] - R[2, 2] + 1, R[1, 0] + R[0, 1], R[2, 0] + R[0, 2]]
    elif dom == 1:
        k1 = [R[1, 0] + R[0, 1], R[1, 1] - R[0, 0] - R[2, 2] + 1, R[2, 1] + R[1, 2]]
    else:
        k1 = [R[2, 0] + R[0, 2], R[2, 1] + R[1, 2], R[2, 2] - R[0, 0] - R[1, 1] + 1]
    sg = _sgn(k[dom])
    v = [k[0] + sg * k1[0], k[1] + sg * k1[1], k[2] + sg * k1[2]]
    nm = np.linalg.norm(v)
    if nm == 0:
        return np.array([1, 0, 0, 0])
    return np.hstack((s, np.dot(np.sqrt(1 - s ** 2) / nm, np.array(v))))


def normalize_angle(angles):
    return [np.arctan2(np.sin(a), np.cos(a)) for a in angles]


def rot2euler(R):
    """Both XYZ-mobile Euler solutions; clamps R[0, 2] into [-1, 1] in place (reference quirk)."""
    th = np.abs(np.abs(R[0, 2]) - 1.0)
    R[0, 2] = min(R[0, 2], 1)
    R[0, 2] = max(R[0, 2], -1)
    if th > 0.0001:
        b1 = np.arcsin(R[0, 2])
        b2 = np.pi - b1
        s1, s2 = np.sign(np.cos(b1)), np.sign(np.cos(b2))
        a1 = np.arctan2(-s1 * R[1][2], s1 * R[2][2])
        g1 = np.arctan2(-s1 * R[0][1], s1 * R[0][0])
        a2 = np.arctan2(-s2 * R[1][2], s2 * R[2][2])
        g2 = np.arctan2(-s2 * R[0][1], s2 * R[0][0])
    else:          # gimbal lock: alpha fixed to 0 / pi
        a1, a2 = 0, np.pi
        b1 = np.arcsin(R[0, 2])
        if b1 > 0:
            b2 = np.pi / 2
            g1 = np.arctan2(R[1][0], R[1][1])
            g2 = np.arctan2(R[1][0], R[1][1]) - a2
        else:
            b2 = -np.pi / 2
            g1 = np.arctan2(-R[1][0], R[1][1])
            g2 = np.arctan2(-R[1][0], R[1][1]) - a2
    return normalize_angle([a1, b1, g1]), normalize_angle([a2, b2, g2])


# ------------------------------------------------------------------------------------------
# value types
# ------------------------------------------------------------------------------------------
class Euler:
    def __init__(self, abg):
        self.abg = abg.abg if isinstance(abg, Euler) else np.asarray(abg) if not isinstance(
            abg, np.ndarray) else abg

    def R(self):
        return RotationMatrix(euler2rot(self.abg))

    def Q(self):
        return Quaternion(rot2quaternion(euler2rot(self.abg)))

    def __str__(self):
        return str(self.abg)


class Quaternion:
    def __init__(self, array):
        self.array = np.array(array)

    def R(self):
        return RotationMatrix(quaternion2rot(self.array))

    def Euler(self):
        e = rot2euler(quaternion2rot(self.array))
        return Euler(e[0]), Euler(e[1])

    def Q(self):
        return self

    def __getitem__(self, item):
        return self.array[item]

    def toarray(self):
        return self.array

    def __str__(self):
        return str(self.array)


class RotationMatrix:
    def __init__(self, m):
        if isinstance(m, RotationMatrix):
            self.array = m.toarray()
        elif isinstance(m, int):
            self.array = np.eye(m)
        else:
            self.array = m if isinstance(m, np.ndarray) else np.array(m)

    def toarray(self):
        return self.array

    def __getitem__(self, item):
        return self.array[item[0], item[1]]

    def inv(self):
        return RotationMatrix(self.array.T)

    def R(self):
        return self

    def Q(self):
        return Quaternion(rot2quaternion(self.array))

    def euler(self):
        e = rot2euler(self.array)
        return Euler(e[0]), Euler(e[1])

    def __str__(self):
        return str(self.array)


def _build(position, orientation):
    T = np.zeros((4, 4))
    T[0:3, 0:3] = orientation.R().toarray()
    T[3, 3] = 1
    T[0:3, 3] = np.array(position).T
    return T


class HomogeneousMatrix:
    """4x4 float64 rigid transform; ``.array`` is the numpy matrix (row-major)."""

    def __init__(self, *args):
        if len(args) == 0:
            self.array = np.eye(4)
        elif len(args) == 1:
            a = args[0]
            if isinstance(a, HomogeneousMatrix):
                self.array = a.toarray()
            elif isinstance(a, np.ndarray):
                self.array = a
            else:
                self.array = np.array(a)
        elif len(args) == 2:
            pos, ori = args
            if not isinstance(pos, np.ndarray):
                pos = np.array(pos.array if hasattr(pos, "array") else pos)
            if isinstance(ori, list):
                ori = Euler(ori)
            if not isinstance(ori, (Euler, Quaternion, RotationMatrix)):
                raise TypeError("orientation must be Euler, Quaternion, RotationMatrix or list")
            self.array = _build(pos, ori)
        else:
            raise TypeError("HomogeneousMatrix takes 0, 1 or 2 arguments")

    def __str__(self):
        return str(self.array)

    def __repr__(self):
        return f"HomogeneousMatrix({self.array!r})"

    def toarray(self):
        return self.array

    def print_nice(self, precision=3):
        print(np.array_str(self.array, precision=precision, suppress_small=True))

    def inv(self):
        return HomogeneousMatrix(np.linalg.inv(self.array))

    def Q(self):
        return Quaternion(rot2quaternion(self.array))

    def R(self):
        return RotationMatrix(self.array[0:3, 0:3])   # a view, as in the reference

    def euler(self):
        return self.R().euler()[0], self.R().euler()[1]

    def pos(self):
        return self.array[0:3, 3]

    def __mul__(self, other):
        if isinstance(other, HomogeneousMatrix):
            return HomogeneousMatrix(np.dot(self.array, other.array))
        return np.dot(self.array, np.asarray(getattr(other, "array", other)))

    def __add__(self, other):
        return HomogeneousMatrix(self.array + other.array)

    def __sub__(self, other):
        return HomogeneousMatrix(self.array - other.array)

    def __getitem__(self, item):
        return self.array[item[0], item[1]]

    def t2v(self, n=2):
        if n == 2:
            return np.array([self.array[0, 3], self.array[1, 3],
                             np.arctan2(self.array[1, 0], self.array[0, 0])])
        th = self.Q().Euler()[0].abg
        return np.array([self.array[0, 3], self.array[1, 3], self.array[2, 3],
                         th[0], th[1], th[2]])


# ------------------------------------------------------------------------------------------
# transform lists (artelib/homogeneousmatrix.py:147-212)
# ------------------------------------------------------------------------------------------
def compute_homogeneous_transforms(df_data):
    """Rows with x, y, z, qx, qy, qz, qw -> HomogeneousMatrix list (quaternion order [w,x,y,z])."""
    out = []
    for i in df_data.index:
        q = [df_data["qw"][i], df_data["qx"][i], df_data["qy"][i], df_data["qz"][i]]
        p = [df_data["x"][i], df_data["y"][i], df_data["z"][i]]
        out.append(HomogeneousMatrix(p, Quaternion(q)))
    return out


def compute_relative_transformations(global_transforms):
    return [global_transforms[i].inv() * global_transforms[i + 1]
            for i in range(len(global_transforms) - 1)]


def compute_global_transformations(transforms_relative, T0, Trobot_gps):
    T = HomogeneousMatrix() if T0 is None else T0
    if Trobot_gps is None:
        Trobot_gps = HomogeneousMatrix()
    out = [T0]
    for Tij in transforms_relative:
        T = T * Tij
        out.append(T)
    return [Ti * Trobot_gps for Ti in out]


def multiply_by_transform(transforms, Trel):
    return [T * Trel for T in transforms]
