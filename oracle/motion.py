"""CPU restatement of the reference's object-motion path.

TEST INFRASTRUCTURE ONLY: tests/ use it to check the product's rt_object_*
(csrc/motion.cpp) bit for bit.  Written from the reference directly
(TD/ = TEST_Dungeonrun/), not from motion.cpp:

* WinMain's key block (TD/WinMain.cpp:186-209) -> Input::set_quat
  (TD/Input.cpp:16-19) -> Object::transform (TD/Object.cpp:14-17) ->
  transform_camera_voxel_device_memory (TD/Camera.cu:254-335);
* VEC4 operators and normalize_Vector (TD/Vector.h:89-124), VEC4::rotate
  (TD/vector.cpp:38-65), vector_norm (TD/vector.cpp:13-26, upper union bytes
  taken as zero, as in np_oracle.rsqrt);
* the device rot_m: set_rotation_matrix copies (TD/Quaternion.cu:4-10,21-25)
  and update_voxel_transform_m_translate_cuda (TD/Camera.cu:188-192), whose
  `w += s * x * d` is taken as nvcc's contracted fma(s * x, d, w).

Host arithmetic is float32 with one rounding per operation, left to right
(MSVC x64 /fp:precise does not contract).  The fma is evaluated exactly with
fractions and rounded once to float32.

Parity unpinned: the reference cannot be run here and ships no recorded
motion, so this restatement is the only check.
"""
from __future__ import annotations

from fractions import Fraction

import numpy as np

from .np_oracle import rsqrt

F = np.float32
TRANSLATE_XYZ, TRANSLATE_X, TRANSLATE_Z = 30, 31, 32   # TD/platform_common.h:15-17
ROTATE_TRI_PY, ROTATE_TRI_NY = 10, 11                  # TD/platform_common.h:19-20
KEY_R, KEY_W, KEY_S, KEY_Q, KEY_E, KEY_T = 1, 2, 4, 8, 16, 32


def _round_f32(v: Fraction) -> F:
    """Round an exact rational to the nearest float32 (ties to even)."""
    f = F(float(v))
    if Fraction(float(f)) == v:
        return f
    g = np.nextafter(f, F(np.inf) if Fraction(float(f)) < v else F(-np.inf))
    da, db = abs(Fraction(float(f)) - v), abs(Fraction(float(g)) - v)
    if da != db:
        return f if da < db else g
    return f if int(np.array([f], F).view(np.uint32)[0]) % 2 == 0 else g


def fma32(a, b, c) -> F:
    return _round_f32(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c)))


class V4:
    """VEC4<float> (TD/Vector.h:65-112): x y z w (w aliases d)."""

    def __init__(self, x, y, z, w):
        self.x, self.y, self.z, self.w = F(x), F(y), F(z), F(w)

    def copy(self):
        return V4(self.x, self.y, self.z, self.w)

    def as_list(self):
        return [self.x, self.y, self.z, self.w]

    def isub(self, r):   # TD/Vector.h:89-94
        self.x = F(F(self.x * self.w) - F(r.x * r.w))
        self.y = F(F(self.y * self.w) - F(r.y * r.w))
        self.z = F(F(self.z * self.w) - F(r.z * r.w))
        self.w = F(1.0)

    def iadd(self, r):   # TD/Vector.h:95-100
        self.x = F(F(self.x * self.w) + F(r.x * r.w))
        self.y = F(F(self.y * self.w) + F(r.y * r.w))
        self.z = F(F(self.z * self.w) + F(r.z * r.w))
        self.w = F(1.0)

    def negate(self):    # TD/Vector.h:105
        self.x, self.y, self.z = -self.x, -self.y, -self.z

    def normalize(self):  # TD/Vector.h:116-124
        s = F(F(F(self.x * self.x) + F(self.y * self.y)) + F(self.z * self.z))
        s = rsqrt(s, 8)
        self.x, self.y, self.z = F(self.x * s), F(self.y * s), F(self.z * s)
        self.w = F(F(1.0) / s)


class Motion:
    """One Object's transform state after Camera::add_object (TD/Camera.cpp:131-134)."""

    def __init__(self, cam_pos, cam_n, cam_u, speed=F(.005)):
        p = [F(v) for v in cam_pos]
        self.n = [F(v) for v in cam_n]
        self.u = [F(v) for v in cam_u]
        self.speed = F(speed)
        self.q = V4(0, 0, 0, 1)                                   # TD/Quaternion.cpp:17-22
        self.rot = [V4(1, 0, 0, 0), V4(0, 1, 0, 0), V4(0, 0, 1, 0)]
        self.drot = [r.copy() for r in self.rot]                  # initialize_CUDA
        self.init_face = V4(-p[0], -p[1], -p[2], 1.0)
        self.cur_face = V4(-p[0], -p[1], -p[2], 1.0)

    def _rotate(self, v: V4, nv, reverse: int):
        """VEC4::rotate (TD/vector.cpp:38-65)."""
        q, R = self.q, self.rot
        if nv is not None:
            ti, tj, tk, tw = q.x, q.y, q.z, q.w
            q.x = F(F(F(F(tj * nv.z) - F(tk * nv.y)) + F(ti * nv.w)) + F(tw * nv.x))
            q.y = F(F(F(F(tk * nv.x) - F(ti * nv.z)) + F(tj * nv.w)) + F(tw * nv.y))
            q.z = F(F(F(F(ti * nv.y) - F(tj * nv.x)) + F(tk * nv.w)) + F(tw * nv.z))
            q.w = F(F(F(F(tw * nv.w) - F(ti * nv.x)) - F(tj * nv.y)) - F(tk * nv.z))
            two, one = F(2), F(1)

            def p2(a, b):
                return F(F(two * a) * b)
            R[0].x = F(F(one - p2(q.y, q.y)) - p2(q.z, q.z))
            R[0].y = F(p2(q.x, q.y) - p2(q.z, q.w))
            R[0].z = F(p2(q.x, q.z) + p2(q.y, q.w))
            R[1].x = F(p2(q.x, q.y) + p2(q.z, q.w))
            R[1].y = F(F(one - p2(q.x, q.x)) - p2(q.z, q.z))
            R[1].z = F(p2(q.y, q.z) - p2(q.x, q.w))
            R[2].x = F(p2(q.x, q.z) - p2(q.y, q.w))
            R[2].y = F(p2(q.y, q.z) + p2(q.x, q.w))
            R[2].z = F(F(one - p2(q.x, q.x)) - p2(q.y, q.y))
        rv = F(reverse)
        tx, ty, tz = F(v.x * rv), F(v.y * rv), F(v.z * rv)
        out = []
        for r in R:
            out.append(F(F(F(tx * r.x) + F(ty * r.y)) + F(tz * r.z)))
        v.x, v.y, v.z = out

    def _device_translate(self, t: V4, scale: int):
        """update_voxel_transform_m_translate_cuda (TD/Camera.cu:188-192), contracted."""
        s = F(scale)
        for r, c in zip(self.drot, (t.x, t.y, t.z)):
            r.w = fma32(F(s * c), t.w, r.w)

    def transform(self, t_vec, select: int):
        """transform_camera_voxel_device_memory (TD/Camera.cu:254-335)."""
        tv = V4(*[F(v) for v in t_vec])
        if select in (TRANSLATE_XYZ, TRANSLATE_X, TRANSLATE_Z):
            self.init_face.isub(tv)
            self._rotate(tv, None, -1)
            for r, c in zip(self.rot, (tv.x, tv.y, tv.z)):
                r.w = F(r.w + F(tv.w * c))
            self._device_translate(tv, 1)
            self.init_face.normalize()
            self.cur_face = self.init_face.copy()
            self._rotate(self.cur_face, None, -1)
            self.cur_face.negate()
        elif select in (ROTATE_TRI_PY, ROTATE_TRI_NY):
            t = self.init_face.copy()
            self._rotate(t, tv, -1)
            self.drot = [r.copy() for r in self.rot]           # set_device_rotation
            t.iadd(self.cur_face)
            for r, c in zip(self.rot, (t.x, t.y, t.z)):
                r.w = F(r.w - F(c * t.w))
            self._device_translate(t, -1)
            t.isub(self.cur_face)
            self.cur_face = t
            self.cur_face.normalize()
            self.cur_face.negate()
        else:
            raise ValueError(f"unknown transform {select}")

    def tick(self, keys: int):
        """TD/WinMain.cpp:186-209 (order R, W, S, Q, E, T)."""
        a, b = F(0.09950371902099893), F(0.9950371902099893)
        if keys & KEY_R:
            self.transform([0.0, a, 0.0, b], ROTATE_TRI_PY)
        if keys & KEY_W:
            self.transform([*self.n, self.speed], TRANSLATE_Z)
        if keys & KEY_S:
            self.transform([*self.n, -self.speed], TRANSLATE_Z)
        if keys & KEY_Q:
            self.transform([*self.u, self.speed], TRANSLATE_X)
        if keys & KEY_E:
            self.transform([*self.u, -self.speed], TRANSLATE_X)
        if keys & KEY_T:
            self.transform([0.0, -a, 0.0, b], ROTATE_TRI_NY)

    def xform(self) -> np.ndarray:
        return np.array([c for r in self.drot for c in r.as_list()], F)

    def host_rot(self) -> np.ndarray:
        return np.array([c for r in self.rot for c in r.as_list()], F)
