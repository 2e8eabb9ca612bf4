"""ctypes binding of oracle/build/liboracle.so (the CPU restatement).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.  The product package never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
FLAG_SHADOW = 4  # ORC_FLAG_SHADOW

LEAF_DTYPE = np.dtype([
    ("x0", "<f4"), ("x1", "<f4"), ("y0", "<f4"), ("y1", "<f4"), ("z0", "<f4"), ("z1", "<f4"),
    ("sx0", "<i8"), ("sy0", "<i8"), ("sz0", "<i8"), ("sx1", "<i8"), ("sy1", "<i8"), ("sz1", "<i8"),
    ("tri", "<i8"),
])
assert LEAF_DTYPE.itemsize == 80

NODE_DTYPE = np.dtype([
    ("x0", "<f4"), ("x1", "<f4"), ("y0", "<f4"), ("y1", "<f4"), ("z0", "<f4"), ("z1", "<f4"),
    ("s1", "<f4"), ("s2", "<f4"), ("cut_flag", "<i4"), ("is_leaf", "<i4"),
    ("tri_index", "<i8"), ("left", "<i8"), ("right", "<i8"), ("parent", "<i8"),
    ("l", "<i8"), ("m", "<i8"), ("r", "<i8"),
])
assert NODE_DTYPE.itemsize == 96


class OrcCamera(C.Structure):
    _fields_ = [("w", C.c_int32), ("h", C.c_int32), ("pos", C.c_float * 3),
                ("n", C.c_float * 3), ("u", C.c_float * 3), ("v", C.c_float * 3),
                ("n_mod", C.c_float * 3), ("u_mod", C.c_float * 3), ("v_mod", C.c_float * 3),
                ("pix_w", C.c_float), ("pix_h", C.c_float)]


CNT_INTERIOR, CNT_LEAF, CNT_ACCEPT, CNT_HITPIX, CNT_DESCEND, CNT_MAXSTACK = range(6)

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        P = C.c_void_p
        L.orc_read_ply.argtypes = [C.c_char_p, C.c_int, C.POINTER(P), C.POINTER(C.c_uint32), C.POINTER(P)]
        L.orc_assemble.argtypes = [P, C.c_int64, P, P, C.c_int64, C.POINTER(P), C.POINTER(C.c_uint32), C.POINTER(P)]
        L.orc_free.argtypes = [P]
        L.orc_build_kd.argtypes = [P, C.c_uint32, P]
        L.orc_camera_basis.argtypes = [C.c_int32, C.c_int32, C.c_float, C.c_float, C.c_float, P, P, P,
                                       C.POINTER(OrcCamera)]
        L.orc_film_w.argtypes = [C.c_int32, C.c_int32]
        L.orc_film_w.restype = C.c_float
        L.orc_host_vector_norm.argtypes = [C.c_float]
        L.orc_host_vector_norm.restype = C.c_float
        L.orc_device_inverse_sqrt.argtypes = [C.c_float, C.c_float, C.c_float]
        L.orc_device_inverse_sqrt.restype = C.c_float
        L.orc_scene_create.argtypes = [P, P, C.c_uint32, P, C.POINTER(OrcCamera)]
        L.orc_scene_create.restype = P
        L.orc_scene_destroy.argtypes = [P]
        L.orc_render.argtypes = [P, P, C.c_int, C.c_int32, C.c_int32, P, P, P, C.c_int]
        L.orc_render_ex.argtypes = [P, P, C.c_int, C.c_int, C.c_int32, C.c_int32, P, P, P, C.c_int]
        L.orc_primary_ray.argtypes = [C.POINTER(OrcCamera), C.c_int32, C.c_int32, P]
        L.orc_phong.argtypes = [P, P, P, P]
        L.orc_phong.restype = C.c_uint32
        L.orc_window_frame.argtypes = [P, P, P, C.c_int64, P]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return C.c_void_p(a.ctypes.data)


def _take(ptr, count, dtype):
    if count == 0:
        lib().orc_free(ptr)
        return np.zeros(0, dtype=dtype)
    buf = (C.c_char * (count * np.dtype(dtype).itemsize)).from_address(ptr.value)
    arr = np.frombuffer(buf, dtype=dtype).copy()
    lib().orc_free(ptr)
    return arr


def read_ply(path: str, mode: int):
    """Restated read_ply: returns (points9 [ntri,9] f32, leafs LEAF_DTYPE)."""
    pts, lf, n = C.c_void_p(), C.c_void_p(), C.c_uint32()
    rc = lib().orc_read_ply(path.encode(), mode, C.byref(pts), C.byref(n), C.byref(lf))
    if rc != 0:
        raise RuntimeError(f"orc_read_ply({path}) failed: {rc}")
    return _take(pts, 9 * n.value, np.float32).reshape(-1, 9), _take(lf, n.value, LEAF_DTYPE)


def assemble(verts: np.ndarray, arity: np.ndarray, idx: np.ndarray):
    verts = np.ascontiguousarray(verts, dtype=np.float32)
    arity = np.ascontiguousarray(arity, dtype=np.int32)
    idx = np.ascontiguousarray(idx, dtype=np.int32)
    pts, lf, n = C.c_void_p(), C.c_void_p(), C.c_uint32()
    rc = lib().orc_assemble(_ptr(verts), len(verts), _ptr(arity), _ptr(idx), len(arity),
                            C.byref(pts), C.byref(n), C.byref(lf))
    if rc != 0:
        raise RuntimeError(f"orc_assemble failed: {rc}")
    return _take(pts, 9 * n.value, np.float32).reshape(-1, 9), _take(lf, n.value, LEAF_DTYPE)


def build_kd(leafs: np.ndarray) -> np.ndarray:
    leafs = np.ascontiguousarray(leafs, dtype=LEAF_DTYPE)
    n = len(leafs)
    nodes = np.zeros(max(2 * n - 1, 1), dtype=NODE_DTYPE)
    rc = lib().orc_build_kd(_ptr(leafs), n, _ptr(nodes))
    if rc != 0:
        raise RuntimeError(f"orc_build_kd failed: {rc}")
    return nodes


def film_w(w: int, h: int) -> float:
    return float(np.float32(lib().orc_film_w(w, h)))


def camera(w, h, f_w=None, f_h=0.024, focal=0.055, pos=(0.0, 0.1, -1.0),
           look_at=(0.0, 0.1, 0.0), up=(0.0, 1.0, 0.0)) -> OrcCamera:
    """Camera::Camera with the WinMain defaults (TD/WinMain.cpp:69-74)."""
    if f_w is None:
        f_w = film_w(w, h)
    cam = OrcCamera()
    p = np.asarray(pos, np.float32); la = np.asarray(look_at, np.float32); u = np.asarray(up, np.float32)
    lib().orc_camera_basis(w, h, np.float32(f_w), np.float32(f_h), np.float32(focal),
                           _ptr(p), _ptr(la), _ptr(u), C.byref(cam))
    return cam


class Scene:
    """Trixel + Camera device state restated on the host."""

    def __init__(self, points9, rad3, nodes, cam: OrcCamera):
        self.points9 = np.ascontiguousarray(points9, dtype=np.float32)
        self.rad3 = np.ascontiguousarray(rad3, dtype=np.float32)
        self.ntri = len(self.points9)
        self.nodes = None if nodes is None else np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
        self.cam = cam
        self._h = lib().orc_scene_create(_ptr(self.points9), _ptr(self.rad3), self.ntri,
                                         None if self.nodes is None else _ptr(self.nodes),
                                         C.byref(cam))

    def render(self, mode=0, xform=None, rows=None, nthreads=0, want_hit=True, shadow=False):
        """shadow=True: one shadow ray per hit (ORC_FLAG_SHADOW, KD only)."""
        w, h = self.cam.w, self.cam.h
        argb = np.zeros(w * h, np.uint32)
        hit = np.full(w * h, -1, np.int64) if want_hit else None
        cnt = np.zeros(6, np.uint64)
        r0, r1 = (0, h) if rows is None else rows
        X = None if xform is None else np.ascontiguousarray(xform, np.float32)
        rc = lib().orc_render_ex(self._h, None if X is None else _ptr(X), mode, FLAG_SHADOW if shadow else 0,
                                 r0, r1, _ptr(argb), None if hit is None else _ptr(hit), _ptr(cnt), nthreads)
        if rc != 0:
            raise RuntimeError(f"orc_render failed: {rc}")
        return argb, hit, cnt

    def close(self):
        if self._h:
            lib().orc_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Window:
    """The reference's persistent window buffer (orc_window_frame): zero at
    first (TD/Camera.cu:98); frame() returns what the window shows for one
    frame's steady-state render (clean argb, hit)."""

    def __init__(self, npix: int):
        self.buf = np.zeros(npix, np.uint32)

    def frame(self, clean: np.ndarray, hit: np.ndarray) -> np.ndarray:
        clean = np.ascontiguousarray(clean, np.uint32)
        hit = np.ascontiguousarray(hit, np.int64)
        out = np.zeros_like(self.buf)
        lib().orc_window_frame(_ptr(self.buf), _ptr(clean), _ptr(hit), len(self.buf), _ptr(out))
        return out


def default_rad(ntri: int) -> np.ndarray:
    """Material of TD/WinMain.cpp:117-121."""
    r = np.empty((ntri, 3), np.float32)
    r[:, 0] = np.float32(0.1); r[:, 1] = np.float32(0.55); r[:, 2] = np.float32(0.2)
    return r
