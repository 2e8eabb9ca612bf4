"""ctypes binding of librt_mi355x.so (include/rt_mi355x.h).

The library is built in-tree by ``python -m cpp_cuda_raytracer_dev_amd.build``
(or ``__graft_entry__.build()``).  There is no fallback: if the shared object
is missing, importing the renderer raises, so a GPU run can never silently
use anything but the HIP kernels.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "librt_mi355x.so")
DEFAULT_LIB_PATH = LIB_PATH

RT_OK = 0
RT_MODE_KD = 0
RT_MODE_FLAT = 1
RT_FLAG_WRITE_HIT = 1
RT_FLAG_COUNT = 2
RT_FLAG_SHADOW = 4
RT_FLAG_FRAME_OUT = 8
RT_OPT_KERNEL = 1
RT_OPT_TILE_ORDER = 2
RT_OPT_RAYS = 3
RT_OPT_ITEMS = 4
RT_OPT_COARSE = 5
RT_OPT_SHADOW_ORDER = 6
RT_OPT_FLAT = 7
RT_OPT_RAYS_USED = 8
RT_OPT_SPLIT_USED = 9
RT_OPT_FAST_USED = 12
RT_OPT_ORDER_RESTORES = 13
RT_OPT_FINE_TILES = 14
RT_SCENE_ORDER = 1
RT_SCENE_TREELET_HEIGHT = 2
RT_SCENE_TWO_LEVEL_DEPTH = 3
RT_OPT_DEBUG = 100
RT_OPT_POOL_CAP = 101
RT_COMM_ID_BYTES = 128

LEAF_AABB_DTYPE = np.dtype([("x0", "<f4"), ("x1", "<f4"), ("y0", "<f4"), ("y1", "<f4"),
                            ("z0", "<f4"), ("z1", "<f4"), ("tri", "<i8")])
assert LEAF_AABB_DTYPE.itemsize == 32

KD_NODE_DTYPE = np.dtype([
    ("x0", "<f4"), ("x1", "<f4"), ("y0", "<f4"), ("y1", "<f4"), ("z0", "<f4"), ("z1", "<f4"),
    ("s1", "<f4"), ("s2", "<f4"), ("cut_flag", "<i4"), ("is_leaf", "<i4"),
    ("tri_index", "<i8"), ("left", "<i8"), ("right", "<i8"), ("parent", "<i8"),
])
assert KD_NODE_DTYPE.itemsize == 72


class RtCameraBasis(C.Structure):
    _fields_ = [("n", C.c_float * 3), ("u", C.c_float * 3), ("v", C.c_float * 3),
                ("n_mod", C.c_float * 3), ("u_mod", C.c_float * 3), ("v_mod", C.c_float * 3),
                ("pix_w", C.c_float), ("pix_h", C.c_float)]


class RtFrameGeometry(C.Structure):
    _fields_ = [("w", C.c_int32), ("h", C.c_int32), ("n_mod", C.c_float * 3), ("u_mod", C.c_float * 3),
                ("v_mod", C.c_float * 3), ("root_box", C.c_float * 6), ("root_is_leaf", C.c_int32),
                ("kernel", C.c_int32), ("rays", C.c_int32), ("coarse", C.c_int32), ("debug", C.c_int32)]


class RtTile(C.Structure):
    _fields_ = [("nranks", C.c_int32), ("rank", C.c_int32)]


RT_LOOP_MAX_BUF = 8
RT_LOOP_MAX_LANES = 4
RT_LOOP_MULTIFRAME = -1


class RtFrameLoop(C.Structure):
    _fields_ = [("xform", C.c_void_p), ("mode", C.c_uint32), ("flags", C.c_uint32), ("tile", RtTile),
                ("nbuf", C.c_int32), ("d_local", C.c_void_p * RT_LOOP_MAX_BUF),
                ("d_scratch", C.c_void_p * RT_LOOP_MAX_BUF), ("d_frame", C.c_void_p * RT_LOOP_MAX_BUF),
                ("render_stream", C.c_void_p), ("comm_stream", C.c_void_p), ("event_every", C.c_int32),
                ("inflight", C.c_int32), ("xforms", C.c_void_p), ("nxforms", C.c_int32)]


class RtError(RuntimeError):
    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} failed ({code}): {msg}")
        self.code = code


# name -> (restype, argtypes); every symbol include/rt_mi355x.h declares.
_P = C.c_void_p
SIGNATURES = {
    "rt_read_ply": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(_P), C.POINTER(C.c_uint32), C.POINTER(_P)]),
    "rt_mesh_assemble": (C.c_int, [_P, C.c_int64, _P, _P, C.c_int64, C.POINTER(_P), C.POINTER(C.c_uint32),
                                   C.POINTER(_P)]),
    "rt_host_free": (None, [_P]),
    "rt_kd_build": (C.c_int, [_P, C.c_uint32, _P, C.c_int]),
    "rt_kd_build_gpu": (C.c_int, [C.c_int, _P, C.c_uint32, _P, _P]),
    "rt_scene_build_kd": (C.c_int, [_P, _P, C.c_uint32, _P]),
    "rt_scene_read_kd": (C.c_int, [_P, _P, C.c_uint64]),
    "rt_camera_basis": (C.c_int, [C.c_int32, C.c_int32, C.c_float, C.c_float, C.c_float, _P, _P, _P,
                                  C.POINTER(RtCameraBasis)]),
    "rt_film_w": (C.c_float, [C.c_int32, C.c_int32]),
    "rt_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "rt_scene_create": (C.c_int, [C.c_int, _P, _P, C.c_uint32, C.POINTER(_P)]),
    "rt_scene_set_kd": (C.c_int, [_P, _P, C.c_uint64]),
    "rt_scene_set_option": (C.c_int, [_P, C.c_int32, C.c_int32]),
    "rt_scene_get_option": (C.c_int, [_P, C.c_int32, C.POINTER(C.c_int32)]),
    "rt_camera_create": (C.c_int, [C.c_int, C.c_int32, C.c_int32, C.c_float, C.c_float, C.c_float, _P, _P, _P,
                                   C.POINTER(_P)]),
    "rt_camera_add_object": (C.c_int, [_P, _P]),
    "rt_render": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, C.POINTER(RtTile), _P]),
    "rt_render_into": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, C.POINTER(RtTile), _P, _P, _P]),
    "rt_render_display": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, C.POINTER(RtTile), _P, _P, _P, _P]),
    "rt_tile_packed_pixels": (C.c_int64, [C.c_int32, C.c_int32, C.c_int32]),
    "rt_unpack_bands": (C.c_int, [C.c_int, C.c_int32, C.c_int32, C.c_int32, _P, _P, _P]),
    "rt_comm_available": (C.c_int, []),
    "rt_comm_unique_id": (C.c_int, [_P]),
    "rt_comm_create": (C.c_int, [C.c_int, C.c_int32, C.c_int32, _P, C.POINTER(_P)]),
    "rt_comm_gather_frame": (C.c_int, [_P, _P, _P, C.c_uint32, _P, _P, _P, _P]),
    "rt_frame_rect": (C.c_int, [_P, _P, C.c_uint32, C.c_int32, _P]),
    "rt_rect_pixels": (C.c_int64, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P]),
    "rt_pack_rect": (C.c_int, [C.c_int, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P, _P, _P, _P]),
    "rt_unpack_rect": (C.c_int, [C.c_int, C.c_int32, C.c_int32, C.c_int32, _P, _P, _P, _P, _P]),
    "rt_camera_frame_geometry": (C.c_int, [_P, C.POINTER(RtFrameGeometry)]),
    "rt_frame_rect_host": (C.c_int, [C.POINTER(RtFrameGeometry), _P, C.c_uint32, C.c_int32, _P]),
    "rt_pack_rect_host": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P, _P, _P]),
    "rt_unpack_rect_host": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, _P, _P, _P, _P]),
    "rt_comm_info": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "rt_comm_destroy": (None, [_P]),
    "rt_run_frames": (C.c_int, [_P, _P, C.POINTER(RtFrameLoop), C.c_int32, C.POINTER(C.c_int64),
                                C.POINTER(C.c_double), C.POINTER(C.c_int32), C.POINTER(C.c_double)]),
    "rt_read_frame": (C.c_int, [_P, _P, _P]),
    "rt_camera_counters": (C.c_int, [_P, _P, C.c_int]),
    "rt_pinned_alloc": (C.c_int, [C.c_size_t, C.POINTER(_P)]),
    "rt_pinned_free": (None, [_P]),
    "rt_frame_copy_async": (C.c_int, [C.c_int, _P, _P, C.c_int64, _P]),
    "rt_object_create": (C.c_int, [_P, _P, _P, C.c_float, C.POINTER(_P)]),
    "rt_object_transform": (C.c_int, [_P, _P, C.c_int32]),
    "rt_object_tick": (C.c_int, [_P, C.c_uint32]),
    "rt_object_xform": (C.c_int, [_P, _P]),
    "rt_object_state": (C.c_int, [_P, _P, _P, _P, _P]),
    "rt_object_destroy": (None, [_P]),
    "rt_camera_error": (C.c_int, [_P, C.POINTER(C.c_int32), C.c_int]),
    "rt_camera_info": (C.c_int, [_P, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "rt_camera_set_option": (C.c_int, [_P, C.c_int32, C.c_int32]),
    "rt_camera_get_option": (C.c_int, [_P, C.c_int32, C.POINTER(C.c_int32)]),
    "rt_camera_debug_read": (C.c_int64, [_P, _P, C.c_int64]),
    "rt_scene_destroy": (None, [_P]),
    "rt_camera_destroy": (None, [_P]),
    "rt_last_error_string": (C.c_char_p, []),
    "rt_abi_version": (C.c_int, []),
    "rt_build_id": (C.c_char_p, []),
}

_lib = None


def lib() -> C.CDLL:
    """Load the HIP library; raise loudly if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build the HIP extension with "
                "`python -m cpp_cuda_raytracer_dev_amd.build` (there is no CPU fallback)")
        # torch bundles its own libamdhip64.so.7 (same soname as /opt/rocm's).
        # Whichever loads first serves the whole process, and torch cannot
        # initialise its devices on the other one. So load torch's runtime
        # first, and let this library bind to it.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if os.path.abspath(LIB_PATH) == DEFAULT_LIB_PATH:
            # build provenance: the library must have been built from this
            # tree's sources and flags (experiment variants are exempt)
            from . import build
            want, got = build.source_id(), L.rt_build_id().decode()
            if got != want:
                raise ImportError(f"{LIB_PATH} was built from other sources (build id {got[:16]}, this tree "
                                  f"{want[:16]}): rebuild with `python -m cpp_cuda_raytracer_dev_amd.build`")
        _lib = L
    return _lib


def build_id() -> str:
    """The loaded library's build id (SHA-256 of its sources and flags)."""
    return lib().rt_build_id().decode()


def check(fn: str, code: int) -> int:
    if code != RT_OK:
        msg = lib().rt_last_error_string()
        raise RtError(fn, code, msg.decode() if msg else "")
    return code


def call(fn: str, *args) -> int:
    return check(fn, getattr(lib(), fn)(*args))


def ptr(a) -> C.c_void_p:
    """Address of a contiguous numpy array or a torch tensor (host or device)."""
    if a is None:
        return C.c_void_p(None)
    if isinstance(a, np.ndarray):
        assert a.flags["C_CONTIGUOUS"]
        return C.c_void_p(a.ctypes.data)
    return C.c_void_p(a.data_ptr())  # torch.Tensor


def take_host(p: C.c_void_p, count: int, dtype) -> np.ndarray:
    """Copy a library-allocated host array into numpy and free it."""
    dtype = np.dtype(dtype)
    if count == 0 or not p.value:
        if p.value:
            lib().rt_host_free(p)
        return np.zeros(0, dtype=dtype)
    buf = (C.c_char * (count * dtype.itemsize)).from_address(p.value)
    out = np.frombuffer(buf, dtype=dtype).copy()
    lib().rt_host_free(p)
    return out
