"""Host-side mirror of the reference's construction API over the C ABI.

Same names, argument meaning and error behaviour as the reference classes
(TD/ = TEST_Dungeonrun/):

* ``read_ply``           TD/read_ply.cpp:13        -> rt_read_ply
* ``Trixel``             TD/Trixel.h:39-478        -> rt_scene_* / rt_kd_build
* ``Camera``             TD/Camera.h:15-97         -> rt_camera_*
* ``Object``             TD/Object.h:10-19         -> Trixel + Quaternion + motion
* ``Quaternion``         TD/Quaternion.h:5-24      (rot_m only; identity)
* ``Input``              TD/Input.h:3-15           (t_vec of a transform)
* ``ObjectMotion``       TD/Camera.cu:254-335      -> rt_object_* (keyboard transforms)

The frame semantics are the steady state of the reference's loop
(TD/WinMain.cpp:212-237): ``Object.render`` runs the fused bg-fill ->
intersect -> Phong kernel, ``Camera.color_pixels`` copies the u32 frame to
``Camera.h_color`` (the D2H of TD/Camera.cu:84).  Status codes follow the
reference (0 = success); failures of the device path raise ``RtError``.
"""
from __future__ import annotations

import ctypes as C
import sys

import numpy as np

from . import _lib
from ._lib import (KD_NODE_DTYPE, LEAF_AABB_DTYPE, RT_FLAG_COUNT, RT_FLAG_FRAME_OUT, RT_FLAG_SHADOW, RT_FLAG_WRITE_HIT,
                   RT_MODE_FLAT, RT_MODE_KD)

SET_COLOR_TAG = 1      # TD/Camera.h:13
PHONG_COLOR_TAG = 2    # TD/Camera.h:14
TRIXEL_OBJECT_TAG = 0  # TD/Object.h:3
BACKGROUND_ARGB = 0x00F08200  # TD/Camera.cpp:72
TRANSLATE_XYZ, TRANSLATE_X, TRANSLATE_Z = 30, 31, 32  # TD/platform_common.h:15-17
ROTATE_TRI_PY, ROTATE_TRI_NY = 10, 11                 # TD/platform_common.h:19-20
#: Held-key bits of ObjectMotion.tick / Object.key_tick (TD/WinMain.cpp:186-209).
KEY_R, KEY_W, KEY_S, KEY_Q, KEY_E, KEY_T = 1, 2, 4, 8, 16, 32
CAM_SPEED = np.float32(.005)  # TD/WinMain.cpp:170


def _finalize(owner) -> None:
    """__del__ of a handle owner: close it, unless the interpreter is shutting
    down.  Then the HIP runtime (and a profiler's tool library) may already be
    finalising, and releasing device memory from a finaliser can fault
    (a SIGSEGV in __cxa_finalize after bench.py's line
    under rocprofv3); the process's exit returns the memory anyway.  Owners
    close their handles explicitly (bench.py, smoke(), the tests' scenes)."""
    if sys.is_finalizing():
        return
    try:
        owner.close()
    except Exception:
        pass


#: Material of every triangle in the reference demo (TD/WinMain.cpp:117-121).
DEFAULT_RAD = (np.float32(0.1), np.float32(0.55), np.float32(0.2))


def read_ply(file_name: str, mode: int):
    """read_ply(file_name, mode) -> (points [ntri, 9] f32, num_tri, kd_leafs).

    mode: 0 "x y z", 1 "x y z confidence intensity", 2 "x y z nx ny nz"
    (TD/WinMain.cpp:93-109).  Headerless "[ply] nv nf" files are accepted.
    """
    pts, leafs, n = C.c_void_p(), C.c_void_p(), C.c_uint32()
    _lib.call("rt_read_ply", file_name.encode(), mode, C.byref(pts), C.byref(n), C.byref(leafs))
    points = _lib.take_host(pts, 9 * n.value, np.float32).reshape(-1, 9)
    return points, n.value, _lib.take_host(leafs, n.value, LEAF_AABB_DTYPE)


def assemble_mesh(verts: np.ndarray, faces) -> tuple:
    """read_ply's face assembly for an in-memory indexed mesh.

    faces: an [nf, 3] or [nf, 4] int array, or a list of 3/4-element faces.
    Returns (points [ntri, 9], num_tri, kd_leafs) like ``read_ply``.
    """
    verts = np.ascontiguousarray(verts, np.float32).reshape(-1, 3)
    if isinstance(faces, np.ndarray) and faces.ndim == 2:
        arity = np.full(len(faces), faces.shape[1], np.int32)
        idx = np.ascontiguousarray(faces, np.int32).reshape(-1)
    else:
        arity = np.array([len(f) for f in faces], np.int32)
        idx = np.array([i for f in faces for i in f], np.int32)
    pts, leafs, n = C.c_void_p(), C.c_void_p(), C.c_uint32()
    _lib.call("rt_mesh_assemble", _lib.ptr(verts), len(verts), _lib.ptr(arity), _lib.ptr(idx), len(arity),
              C.byref(pts), C.byref(n), C.byref(leafs))
    points = _lib.take_host(pts, 9 * n.value, np.float32).reshape(-1, 9)
    return points, n.value, _lib.take_host(leafs, n.value, LEAF_AABB_DTYPE)


def kd_build(kd_leafs: np.ndarray, nthreads: int = 0) -> np.ndarray:
    """set_sorted_voxels + create_kd as one call: the BFS node array (KD_NODE_DTYPE)."""
    leafs = np.ascontiguousarray(kd_leafs, LEAF_AABB_DTYPE)
    nodes = np.zeros(max(2 * len(leafs) - 1, 1), KD_NODE_DTYPE)
    _lib.call("rt_kd_build", _lib.ptr(leafs), len(leafs), _lib.ptr(nodes), nthreads)
    return nodes


def kd_build_gpu(kd_leafs: np.ndarray, device: int = 0, stream=None) -> np.ndarray:
    """rt_kd_build_gpu: the same node array as ``kd_build``, built on a GPU."""
    leafs = np.ascontiguousarray(kd_leafs, LEAF_AABB_DTYPE)
    nodes = np.zeros(max(2 * len(leafs) - 1, 1), KD_NODE_DTYPE)
    s = C.c_void_p(stream) if isinstance(stream, int) else C.c_void_p(None)
    _lib.call("rt_kd_build_gpu", device, _lib.ptr(leafs), len(leafs), _lib.ptr(nodes), s)
    return nodes


def film_w(w: int, h: int) -> float:
    """WinMain's film width ((float)w/h)*.024f (TD/WinMain.cpp:29,69-70)."""
    return float(np.float32(_lib.lib().rt_film_w(w, h)))


def camera_basis(w, h, f_w, f_h, focal, pos, look_at, up) -> dict:
    b = _lib.RtCameraBasis()
    f = lambda v: np.ascontiguousarray(v, np.float32)  # noqa: E731
    p, la, u = f(pos), f(look_at), f(up)
    _lib.call("rt_camera_basis", w, h, np.float32(f_w), np.float32(f_h), np.float32(focal),
              _lib.ptr(p), _lib.ptr(la), _lib.ptr(u), C.byref(b))
    return {k: np.array(getattr(b, k)[:], np.float32) for k in ("n", "u", "v", "n_mod", "u_mod", "v_mod")} | {
        "pix_w": np.float32(b.pix_w), "pix_h": np.float32(b.pix_h)}


class Quaternion:
    """The object transform the hot kernel reads (d_rot_m, TD/Trixel.cu:60-66).

    ``rot_m`` rows are (i, j, k, w) for x, y, z: a 3x3 rotation plus the
    translation in column w.  Identity at construction (TD/Quaternion.cpp:16-23).
    """

    def __init__(self):
        self.rot_m = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 0]], np.float32)

    def xform(self) -> np.ndarray:
        return np.ascontiguousarray(self.rot_m, np.float32).reshape(12)


class Input:
    """TD/Input.h:3-15 without the Win32 buttons: ``set_quat`` stores the four
    floats as the transform vector (TD/Input.cpp:16-19)."""

    def __init__(self):
        self.t_vec = np.zeros(4, np.float32)

    def set_vec(self, x, y, z, w):
        self.t_vec = np.array([x, y, z, w], np.float32)

    def set_quat(self, x, y, z, w):
        self.set_vec(x, y, z, w)


class ObjectMotion:
    """An object's motion state (quaternion, host and device rot_m,
    init_face / cur_face) as Camera::add_object sets it up
    (TD/Camera.cpp:131-134) and Object::transform updates it
    (TD/Camera.cu:254-335).  ``xform()`` is the device rot_m the kernel reads."""

    def __init__(self, cam_pos, cam_n, cam_u, cam_speed=CAM_SPEED):
        # keep the arrays alive across the call (ptr() holds only the address)
        p, n, u = (np.array(v, np.float32).reshape(3) for v in (cam_pos, cam_n, cam_u))
        h = C.c_void_p()
        _lib.call("rt_object_create", _lib.ptr(p), _lib.ptr(n), _lib.ptr(u), np.float32(cam_speed), C.byref(h))
        self._h = h

    def transform(self, t_vec, transform_select: int) -> None:
        t = np.ascontiguousarray(t_vec, np.float32).reshape(4)
        _lib.call("rt_object_transform", self._h, _lib.ptr(t), int(transform_select))

    def tick(self, held_keys: int) -> None:
        _lib.call("rt_object_tick", self._h, int(held_keys))

    def xform(self) -> np.ndarray:
        out = np.zeros(12, np.float32)
        _lib.call("rt_object_xform", self._h, _lib.ptr(out))
        return out

    def state(self) -> dict:
        q, r, i, c = (np.zeros(n, np.float32) for n in (4, 12, 4, 4))
        _lib.call("rt_object_state", self._h, _lib.ptr(q), _lib.ptr(r), _lib.ptr(i), _lib.ptr(c))
        return {"quat": q, "rot_m": r, "init_face": i, "cur_face": c}

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            _lib.lib().rt_object_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        _finalize(self)


class Trixel:
    """Triangles (+ KD tree) resident on one device (TD/Trixel.h:39-478)."""

    def __init__(self, num_t: int, points_data: np.ndarray, color_data=None, device: int = 0):
        points = np.ascontiguousarray(points_data, np.float32).reshape(-1, 9)[:num_t]
        if len(points) != num_t:
            raise ValueError("points_data holds fewer than num_t triangles")
        if color_data is None:
            rad = np.empty((num_t, 3), np.float32)
            rad[:] = DEFAULT_RAD
        else:
            rad = np.ascontiguousarray(color_data, np.float32).reshape(-1, 3)[:num_t]
        self.num_trixels = num_t
        self.num_voxels = 2 * num_t - 1
        self.device = device
        self.h_points_init_data = points
        self.rad = rad
        self._leafs = None
        self.h_nodes = None
        h = C.c_void_p()
        _lib.call("rt_scene_create", device, _lib.ptr(points), _lib.ptr(rad), num_t, C.byref(h))
        self._h = h

    def set_sorted_voxels(self, voxel_list: np.ndarray, num_leaf_voxels: int) -> int:
        """TD/Trixel.h:386-473: keeps the leaf AABBs for create_kd."""
        if num_leaf_voxels == 0:
            return 0
        self._leafs = np.ascontiguousarray(voxel_list, LEAF_AABB_DTYPE)[:num_leaf_voxels].copy()
        return 0

    def create_kd(self, nthreads: int = 0, on_device: bool = False) -> int:
        """TD/Trixel.h:135-385: -12 if set_sorted_voxels was not called.
        on_device: build on the scene's GPU (rt_scene_build_kd; same nodes)."""
        if self._leafs is None:
            return -12
        if on_device:
            _lib.call("rt_scene_build_kd", self._h, _lib.ptr(self._leafs), len(self._leafs), None)
            self.h_nodes = None
        else:
            self.h_nodes = kd_build(self._leafs, nthreads)
            _lib.call("rt_scene_set_kd", self._h, _lib.ptr(self.h_nodes), len(self.h_nodes))
        self._leafs = None  # the reference frees the sorted lists (TD/Trixel.h:381-383)
        return 0

    def read_kd_nodes(self) -> np.ndarray:
        """The scene's node array, copied back from the device."""
        nodes = np.zeros(2 * self.num_trixels - 1, KD_NODE_DTYPE)
        _lib.call("rt_scene_read_kd", self._h, _lib.ptr(nodes), len(nodes))
        return nodes

    def set_kd_nodes(self, nodes: np.ndarray) -> int:
        """Upload an already built node array (e.g. cached on disk)."""
        self.h_nodes = np.ascontiguousarray(nodes, KD_NODE_DTYPE)
        _lib.call("rt_scene_set_kd", self._h, _lib.ptr(self.h_nodes), len(self.h_nodes))
        return 0

    def set_option(self, key: int, value: int) -> None:
        """Scene layout knobs (_lib.RT_SCENE_ORDER, _lib.RT_SCENE_TREELET_HEIGHT); frames are identical."""
        _lib.call("rt_scene_set_option", self._h, key, value)

    def get_option(self, key: int) -> int:
        v = C.c_int32()
        _lib.call("rt_scene_get_option", self._h, key, C.byref(v))
        return v.value

    def intersect_trixels(self, c: "Camera", q: Quaternion = None, m: int = RT_MODE_KD, flags: int = 0,
                          stream=None) -> int:
        """TD/Trixel.h:474-476.  Unlike the reference, ``m`` selects KD (0) or flat (1)."""
        return c._render(self, q, m, flags, stream)

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            _lib.lib().rt_scene_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        _finalize(self)


class Object:
    """A Trixel plus its own transform (TD/Object.h:10-19)."""

    def __init__(self, x: Trixel, q: Quaternion = None):
        self.object_tag = TRIXEL_OBJECT_TAG
        self.trixel_list = x
        self.quat = q if q is not None else Quaternion()
        self.motion = None  # set by Camera.add_object

    def getTag(self) -> int:  # noqa: N802 (reference name)
        return self.object_tag

    def render(self, c: "Camera", mode: int = RT_MODE_KD, flags: int = 0, stream=None) -> int:
        """Object::render (TD/Object.cpp:10-12)."""
        return self.trixel_list.intersect_trixels(c, self.quat, mode, flags, stream)

    def _moved(self) -> int:
        if self.motion is None:
            raise _lib.RtError("Object.transform", -5, "add the object to a camera first")
        self.quat.rot_m = self.motion.xform().reshape(3, 4)
        return 0

    def transform(self, dq: Input, transform_select: int) -> int:
        """Object::transform (TD/Object.cpp:14-17); needs Camera.add_object first."""
        if self.motion is None:
            return self._moved()
        self.motion.transform(dq.t_vec, transform_select)
        return self._moved()

    def key_tick(self, held_keys: int) -> int:
        """One input tick of TD/WinMain.cpp:186-209 with KEY_* bits held."""
        if self.motion is None:
            return self._moved()
        self.motion.tick(held_keys)
        return self._moved()


class Camera:
    """Camera (TD/Camera.h:15-97): rays, frame buffer, camera-relative scene data."""

    def __init__(self, r_w, r_h, f_w, f_h, fclen, p_x, p_y, p_z, la_x, la_y, la_z, up_x, up_y, up_z,
                 device: int = 0):
        self.res = (int(r_w), int(r_h))
        self.pos = np.array([p_x, p_y, p_z], np.float32)
        self.la = np.array([la_x, la_y, la_z], np.float32)
        self.up = np.array([up_x, up_y, up_z], np.float32)
        self.device = device
        self.o_prop = camera_basis(r_w, r_h, f_w, f_h, fclen, self.pos, self.la, self.up)
        self.background_color = BACKGROUND_ARGB
        self.cam_speed = CAM_SPEED
        self.object_list = []
        h = C.c_void_p()
        _lib.call("rt_camera_create", device, int(r_w), int(r_h), np.float32(f_w), np.float32(f_h),
                  np.float32(fclen), _lib.ptr(self.pos), _lib.ptr(self.la), _lib.ptr(self.up), C.byref(h))
        self._h = h
        self.h_color = np.zeros(r_w * r_h, np.uint32)
        self.h_rmi = np.full(r_w * r_h, -1, np.int64)

    @classmethod
    def default(cls, w: int, h: int, device: int = 0) -> "Camera":
        """The WinMain camera (TD/WinMain.cpp:69-74) at w x h."""
        return cls(w, h, film_w(w, h), np.float32(.024), np.float32(.055), 0.0, 0.10, -1.0, 0.0, 0.100, 0.0,
                   0.0, 1.0, 0.0, device=device)

    def add_object(self, new_object: Object) -> int:
        """Camera::add_object (TD/Camera.cpp:118-142)."""
        if new_object.getTag() != TRIXEL_OBJECT_TAG:
            return 0
        self.object_list.append(new_object)
        # the object's transform state starts from the camera's (TD/Camera.cpp:131-134)
        new_object.quat = Quaternion()
        new_object.motion = ObjectMotion(self.pos, self.o_prop["n"], self.o_prop["u"], self.cam_speed)
        _lib.call("rt_camera_add_object", self._h, new_object.trixel_list._h)
        return 0

    def _render(self, t: Trixel, q, mode, flags, stream) -> int:
        xf = (q if q is not None else Quaternion()).xform()
        s = C.c_void_p(stream) if isinstance(stream, int) else C.c_void_p(None)
        _lib.call("rt_render", self._h, _lib.ptr(xf), mode, flags, None, s)
        self._last_flags = flags
        return 0

    def render_into(self, argb, hit=None, xform=None, mode=RT_MODE_KD, flags=0, tile=None, stream=None) -> int:
        """Render into caller-owned device buffers (torch tensors or raw pointers)."""
        xf = np.ascontiguousarray(xform if xform is not None else Quaternion().xform(), np.float32)
        t = None if tile is None else C.byref(_lib.RtTile(tile[0], tile[1]))
        s = C.c_void_p(stream) if isinstance(stream, int) else C.c_void_p(None)
        a = argb if isinstance(argb, C.c_void_p) else _lib.ptr(argb)
        h = hit if isinstance(hit, C.c_void_p) else _lib.ptr(hit)
        _lib.call("rt_render_into", self._h, _lib.ptr(xf), mode, flags, t, a, h, s)
        return 0

    def render_display(self, clean, display, hit=None, xform=None, mode=RT_MODE_KD, flags=0, tile=None,
                       stream=None) -> int:
        """rt_render_display: the frame the reference's window shows
        (TD/WinMain.cpp:212-237, ghosting under motion).  `clean` (device,
        zeros before the first frame) holds the previous clean frame and
        receives this one; `display` receives the displayed frame."""
        xf = np.ascontiguousarray(xform if xform is not None else Quaternion().xform(), np.float32)
        t = None if tile is None else C.byref(_lib.RtTile(tile[0], tile[1]))
        s = C.c_void_p(stream) if isinstance(stream, int) else C.c_void_p(None)
        _lib.call("rt_render_display", self._h, _lib.ptr(xf), mode, flags, t, _lib.ptr(clean), _lib.ptr(display),
                  _lib.ptr(hit), s)
        return 0

    def color_pixels(self, color_tag_select: int = PHONG_COLOR_TAG) -> int:
        """Camera::color_pixels (TD/Camera.cpp:229): the frame D2H into h_color.

        Shading is fused into ``Object.render``; both tags yield the steady
        state frame (background where no hit, Phong where hit)."""
        want_hit = bool(getattr(self, "_last_flags", 0) & RT_FLAG_WRITE_HIT)
        _lib.call("rt_read_frame", self._h, _lib.ptr(self.h_color), _lib.ptr(self.h_rmi) if want_hit else None)
        return 0

    def set_option(self, key: int, value: int) -> None:
        """Tuning knobs (_lib.RT_OPT_KERNEL, _lib.RT_OPT_TILE_ORDER); frames are identical."""
        _lib.call("rt_camera_set_option", self._h, key, value)

    def get_option(self, key: int) -> int:
        v = C.c_int32()
        _lib.call("rt_camera_get_option", self._h, key, C.byref(v))
        return v.value

    def counters(self, reset: bool = True) -> np.ndarray:
        out = np.zeros(5, np.uint64)
        _lib.call("rt_camera_counters", self._h, _lib.ptr(out), int(reset))
        return out

    def device_error(self, reset: bool = False) -> int:
        """The device error word every render ORs into (rt_camera_error):
        1 stack overflow, 2 item-pool overflow, 4 far-group proof failed."""
        e = C.c_int32()
        _lib.call("rt_camera_error", self._h, C.byref(e), int(reset))
        return e.value

    def frame(self) -> np.ndarray:
        """h_color as [h, w] u32, row 0 = bottom (the DIB is bottom-up)."""
        w, h = self.res
        return self.h_color.reshape(h, w)

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            _lib.lib().rt_camera_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        _finalize(self)


class FrameLoop:
    """rt_run_frames: the frame loop in native code.  `locals_` are the
    render targets (one per buffer set); with `comm` (a NativeFrameGather),
    each frame is gathered to rank 0 on `comm_stream` while the next renders.
    `inflight` > 1 keeps that many frames in flight on the library's own
    render lanes (without comm, len(locals_) must be a multiple of it).
    `xforms` (n x 12): frame k of the loop renders with pose k mod n.
    ``run(n)`` renders n frames and returns (kernel ms mean, timed frames);
    it synchronises the streams before returning."""

    def __init__(self, cam: "Camera", locals_, xform=None, mode: int = RT_MODE_KD, flags: int = 0, tile=None,
                 render_stream=None, comm=None, comm_stream=None, event_every: int = 0, inflight: int = 1,
                 xforms=None):
        n = len(locals_)
        if not 1 <= n <= _lib.RT_LOOP_MAX_BUF:
            raise ValueError(f"FrameLoop: 1..{_lib.RT_LOOP_MAX_BUF} buffer sets")
        self.cam = cam
        self.comm = comm
        self._xf = np.ascontiguousarray(xform if xform is not None else Quaternion().xform(), np.float32)
        a = _lib.RtFrameLoop()
        a.xform = self._xf.ctypes.data
        a.mode, a.flags = mode, flags
        a.tile = _lib.RtTile(*(tile if tile is not None else (0, 0)))
        a.nbuf = n
        for k in range(n):
            a.d_local[k] = _lib.ptr(locals_[k]).value
            if comm is not None:
                a.d_scratch[k] = _lib.ptr(comm.scratch[k]).value
                f = comm.frames[k]
                a.d_frame[k] = _lib.ptr(f).value if f is not None else None
        a.render_stream = render_stream
        a.comm_stream = comm_stream
        a.event_every = event_every
        a.inflight = inflight
        if xforms is not None:  # one pose per frame, cycled (rt_frame_loop.xforms)
            self._xfs = np.ascontiguousarray(np.asarray(xforms, np.float32).reshape(-1, 12))
            a.xforms = self._xfs.ctypes.data
            a.nxforms = len(self._xfs)
        self._a = a
        self._locals = list(locals_)
        self.seq = C.c_int64(0)

    def run(self, nframes: int):
        """-> (kernel ms mean over the timed frames, timed frames, host ms spent enqueueing)."""
        ms, cnt, host = C.c_double(), C.c_int32(), C.c_double()
        _lib.call("rt_run_frames", self.cam._h, self.comm._h if self.comm is not None else None, C.byref(self._a),
                  int(nframes), C.byref(self.seq), C.byref(ms), C.byref(cnt), C.byref(host))
        return ms.value, cnt.value, host.value

    def last_set(self) -> int:
        """The buffer set the last frame used."""
        return (self.seq.value - 1) % self._a.nbuf


def packed_pixels(w: int, h: int, nranks: int) -> int:
    return int(_lib.lib().rt_tile_packed_pixels(w, h, nranks))


def unpack_bands(device: int, w: int, h: int, nranks: int, gathered, frame, stream=None) -> None:
    s = C.c_void_p(stream) if isinstance(stream, int) else C.c_void_p(None)
    _lib.call("rt_unpack_bands", device, w, h, nranks, _lib.ptr(gathered), _lib.ptr(frame), s)


class PinnedFrames:
    """Frame delivery: `count` page-locked host frames
    of `npix` u32 each, filled by stream-ordered D2H copies so the copy of
    frame k overlaps the render of frame k+1 (the reference copies
    synchronously, TD/Camera.cu:84)."""

    def __init__(self, npix: int, count: int = 2):
        self.npix = int(npix)
        self._ptrs = []
        self.frames = []
        for _ in range(count):
            p = C.c_void_p()
            _lib.call("rt_pinned_alloc", C.c_size_t(4 * max(self.npix, 1)), C.byref(p))
            self._ptrs.append(p)
            buf = (C.c_uint32 * max(self.npix, 1)).from_address(p.value)
            self.frames.append(np.frombuffer(buf, dtype=np.uint32)[: self.npix])

    def copy_async(self, k: int, device: int, d_argb, stream=None) -> None:
        """Enqueue the D2H of device frame d_argb into host frame k on `stream`."""
        s = C.c_void_p(stream) if isinstance(stream, int) else C.c_void_p(None)
        _lib.call("rt_frame_copy_async", device, _lib.ptr(d_argb), self._ptrs[k], self.npix, s)

    def close(self) -> None:
        self.frames = []
        for p in self._ptrs:
            _lib.lib().rt_pinned_free(p)
        self._ptrs = []

    def __del__(self):
        _finalize(self)


__all__ = ["read_ply", "assemble_mesh", "kd_build", "film_w", "camera_basis", "Quaternion", "Trixel", "Object",
           "Camera", "PinnedFrames", "packed_pixels", "unpack_bands", "SET_COLOR_TAG", "PHONG_COLOR_TAG", "RT_MODE_KD",
           "RT_MODE_FLAT", "RT_FLAG_WRITE_HIT", "RT_FLAG_COUNT", "RT_FLAG_SHADOW", "RT_FLAG_FRAME_OUT", "BACKGROUND_ARGB", "DEFAULT_RAD"]
