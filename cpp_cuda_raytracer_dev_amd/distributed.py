"""Multi-GPU frame sharding: disjoint screen bands + a gather to rank 0.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm,
"gloo" for the CPU tests).  The scene is replicated on every GPU (built once
per process from the same deterministic inputs).  Rows are cut into bands of
8 and band b belongs to rank b % N, which interleaves the centrally placed
object across ranks.  Each rank renders its bands into a packed buffer of
equal size; rank 0 gathers the N buffers over xGMI and reassembles the frame
with one kernel (rt_unpack_bands).  The reference is single-GPU
(cudaSetDevice(0) everywhere, TD/Trixel.cu:213): this layer is new.
"""
from __future__ import annotations

import numpy as np

BAND = 8  # rows per band; equals the kernels' tile height


def nbands(h: int) -> int:
    return (h + BAND - 1) // BAND


def slots(h: int, nranks: int) -> int:
    return (nbands(h) + nranks - 1) // nranks


def packed_pixels(w: int, h: int, nranks: int) -> int:
    return slots(h, nranks) * BAND * w


def pack_bands_numpy(frame: np.ndarray, w: int, h: int, nranks: int, rank: int, fill=0) -> np.ndarray:
    """The packed buffer rank `rank` renders: slot j holds band rank + j*nranks."""
    out = np.full(packed_pixels(w, h, nranks), fill, dtype=frame.dtype)
    f = frame.reshape(h, w)
    for j in range(slots(h, nranks)):
        b = rank + j * nranks
        if b >= nbands(h):
            break
        y0, y1 = b * BAND, min(h, (b + 1) * BAND)
        out[j * BAND * w:(j * BAND + (y1 - y0)) * w] = f[y0:y1].reshape(-1)
    return out


def unpack_bands_numpy(gathered: np.ndarray, w: int, h: int, nranks: int) -> np.ndarray:
    """Inverse of the per-rank packing for the N buffers back to back."""
    s = slots(h, nranks)
    g = gathered.reshape(nranks, s, BAND, w)
    y = np.arange(h)
    band, r = y // BAND, y % BAND
    return g[band % nranks, band // nranks, r].reshape(-1)


class FrameGather:
    """Rank-0 gather of the packed band buffers (torch tensors on each rank's device).

    collective="gather": torch.distributed.gather (point-to-point sends to the
    root, one xGMI link per peer); "allgather": all_gather_into_tensor.
    """

    def __init__(self, dist, w: int, h: int, device, collective: str = "gather", unpack=None):
        import torch
        self.dist = dist
        self.w, self.h = w, h
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.npk = packed_pixels(w, h, self.world)
        self.collective = collective
        self.device = device
        self.local = torch.zeros(self.npk, dtype=torch.int32, device=device)
        self.gathered = torch.zeros(self.world * self.npk, dtype=torch.int32, device=device) \
            if (self.rank == 0 or collective == "allgather") else None
        self.frame = torch.zeros(w * h, dtype=torch.int32, device=device) if self.rank == 0 else None
        self.unpack = unpack  # callable(gathered, frame) on rank 0; None -> numpy (CPU tests)

    def gather(self) -> None:
        d = self.dist
        if self.collective == "allgather":
            d.all_gather_into_tensor(self.gathered, self.local)
        else:
            parts = list(self.gathered.split(self.npk)) if self.rank == 0 else None
            d.gather(self.local, gather_list=parts, dst=0)
        if self.rank == 0:
            if self.unpack is not None:
                self.unpack(self.gathered, self.frame)
            else:
                import torch
                g = self.gathered.cpu().numpy().view(np.uint32)
                self.frame.copy_(torch.from_numpy(unpack_bands_numpy(g, self.w, self.h, self.world).view(np.int32)))


class NativeFrameGather:
    """The gather through the library's own RCCL communicator (rt_comm_*).

    One rt_comm_gather_frame call per frame enqueues, on the given stream, the
    peers' pack kernel and ncclSend to rank 0, rank 0's N-1 ncclRecv and the
    assembly kernel -- no Python collective per frame.  Only the rectangle
    rt_frame_rect names travels (outside it the frame is provably
    background).  `nbuf` sets of buffers let frame i+1 render while frame i
    is in flight (bench.py pipelines them with events).  The 128-byte RCCL id
    is broadcast with `dist` (any backend)."""

    def __init__(self, dist, w: int, h: int, device, nbuf: int = 2):
        import ctypes as C
        import torch
        from . import _lib
        self.dist = dist
        self.w, self.h = w, h
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.npk = packed_pixels(w, h, self.world)
        self.device = device
        if not _lib.lib().rt_comm_available():
            raise RuntimeError("NativeFrameGather: librccl.so.1 not found (rt_comm_available() == 0)")
        idb = (C.c_uint8 * _lib.RT_COMM_ID_BYTES)()
        if self.rank == 0:
            _lib.call("rt_comm_unique_id", C.cast(idb, C.c_void_p))
        box = [bytes(idb)]
        dist.broadcast_object_list(box, src=0)
        idb = (C.c_uint8 * _lib.RT_COMM_ID_BYTES).from_buffer_copy(box[0])
        self._h = C.c_void_p()
        _lib.call("rt_comm_create", device.index, self.world, self.rank, C.cast(idb, C.c_void_p), C.byref(self._h))
        # scratch: the peers' rectangle parts on rank 0, the send staging elsewhere
        nscr = max(1, (self.world - 1) * self.npk) if self.rank == 0 else self.npk
        self.local = [torch.zeros(self.npk, dtype=torch.int32, device=device) for _ in range(nbuf)]
        self.scratch = [torch.zeros(nscr, dtype=torch.int32, device=device) for _ in range(nbuf)]
        self.frames = [torch.zeros(w * h, dtype=torch.int32, device=device) if self.rank == 0 else None
                       for _ in range(nbuf)]

    def gather(self, k: int, cam, xform, mode: int, stream) -> None:
        """Stream-ordered gather + assembly of buffer set k, rendered by `cam`
        (raytracer.Camera) with (xform, mode); stream: hipStream_t int."""
        import numpy as np
        from . import _lib
        xf = None if xform is None else np.ascontiguousarray(xform, np.float32)
        f = self.frames[k]
        _lib.call("rt_comm_gather_frame", self._h, cam._h, _lib.ptr(xf), mode, _lib.ptr(self.local[k]),
                  _lib.ptr(self.scratch[k]), _lib.ptr(f) if f is not None else None, stream or None)

    def verify(self, cam, xform, mode: int) -> tuple:
        """Every rank must derive the same rectangle (rt_frame_rect) and render
        with the same options, or rank 0's receive sizes would not match the
        peers' sends (RCCL would hang or truncate instead of failing).  All
        ranks exchange theirs (over `dist`) and raise if any differs.  Returns
        the rectangle."""
        from . import _lib
        rect = self.frame_rect(cam, xform, mode)
        opts = tuple(cam.get_option(k) for k in (_lib.RT_OPT_KERNEL, _lib.RT_OPT_RAYS, _lib.RT_OPT_COARSE,
                                                 _lib.RT_OPT_DEBUG, _lib.RT_OPT_TILE_ORDER))
        return verify_agreement(self.dist, self.world, "NativeFrameGather", rect, opts, (self.w, self.h), mode)

    def frame_rect(self, cam, xform, mode: int):
        """rt_frame_rect for this group's size: (x0, x1, b0, b1)."""
        import numpy as np
        from . import _lib
        xf = None if xform is None else np.ascontiguousarray(xform, np.float32)
        rect = np.zeros(4, np.int32)
        _lib.call("rt_frame_rect", cam._h, _lib.ptr(xf), mode, self.world, _lib.ptr(rect))
        return tuple(int(v) for v in rect)

    def info(self) -> tuple:
        """(ranks, rank) the communicator itself reports (rt_comm_info)."""
        import ctypes as C
        from . import _lib
        n, r = C.c_int32(), C.c_int32()
        _lib.call("rt_comm_info", self._h, C.byref(n), C.byref(r))
        return n.value, r.value

    def close(self) -> None:
        from . import _lib
        if self._h:
            _lib.lib().rt_comm_destroy(self._h)
            self._h = None


def verify_agreement(dist, world: int, who: str, rect, opts, size, mode: int) -> tuple:
    """All ranks exchange (rect, options, size, mode) over `dist` and raise
    RuntimeError on every rank if any differs: message sizes are derived on
    each rank, never exchanged, so a disagreement would otherwise hang or
    truncate the point-to-point transfers."""
    mine = (tuple(int(v) for v in rect), tuple(int(v) for v in opts), tuple(size), int(mode))
    every = [None] * world
    dist.all_gather_object(every, mine)
    if any(e != every[0] for e in every):
        raise RuntimeError(f"{who}: ranks disagree on the frame rectangle / camera options: {every}")
    return mine[0]


def frame_geometry(w: int, h: int, basis, root_box, root_is_leaf: bool = False, kernel: int = 3, rays: int = 0,
                   coarse: int = 8, debug: int = 0):
    """rt_frame_geometry from host-side inputs: `basis` the camera basis
    (raytracer.camera_basis's dict, or an RtCameraBasis), `root_box` the root node's box minus the camera
    position (x0, x1, y0, y1, z0, z1; float32 subtractions)."""
    from . import _lib
    get = (lambda k: basis[k]) if isinstance(basis, dict) else (lambda k: getattr(basis, k))  # noqa: E731
    g = _lib.RtFrameGeometry()
    g.w, g.h = w, h
    for k in range(3):
        g.n_mod[k], g.u_mod[k], g.v_mod[k] = get("n_mod")[k], get("u_mod")[k], get("v_mod")[k]
    for k in range(6):
        g.root_box[k] = float(root_box[k])
    g.root_is_leaf = int(bool(root_is_leaf))
    g.kernel, g.rays, g.coarse, g.debug = kernel, rays, coarse, debug
    return g


def frame_rect_host(geom, xform, mode: int, nranks: int) -> tuple:
    """rt_frame_rect_host: (x0, x1, b0, b1), as rt_frame_rect derives it for a
    camera with this geometry."""
    import ctypes as C
    from . import _lib
    xf = None if xform is None else np.ascontiguousarray(xform, np.float32)
    rect = np.zeros(4, np.int32)
    _lib.call("rt_frame_rect_host", C.byref(geom), _lib.ptr(xf), mode, nranks, _lib.ptr(rect))
    return tuple(int(v) for v in rect)


class HostRectGather:
    """The rectangle gather of rt_comm_gather_frame (csrc/comm.cpp) over host
    buffers and any torch.distributed backend (gloo on CPU): every rank
    derives the rectangle from the same geometry (rt_frame_rect_host, no
    exchange); a peer packs its slots' rows inside it (rt_pack_rect_host) and
    sends exactly rt_rect_pixels(w, h, N, rank, rect) u32 to rank 0; rank 0
    receives the peers' parts in rank order 1..N-1, back to back, and
    assembles the frame from its own packed buffer, those parts and the
    background (rt_unpack_rect_host).  The same protocol as the RCCL path,
    point to point, sizes derived rather than exchanged."""

    def __init__(self, dist, w: int, h: int, geom, xform, mode: int, opts=()):
        self.dist = dist
        self.w, self.h = w, h
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.rect = frame_rect_host(geom, xform, mode, self.world)
        self.opts = tuple(opts) or (geom.kernel, geom.rays, geom.coarse, geom.debug)
        self.mode = mode

    def verify(self) -> tuple:
        return verify_agreement(self.dist, self.world, "HostRectGather", self.rect, self.opts, (self.w, self.h),
                                self.mode)

    def part_pixels(self, rank: int) -> int:
        from . import _lib
        r = np.ascontiguousarray(self.rect, np.int32)
        n = int(_lib.lib().rt_rect_pixels(self.w, self.h, self.world, rank, _lib.ptr(r)))
        if n < 0:
            raise RuntimeError(f"rt_rect_pixels failed for rank {rank}")
        return n

    def gather(self, local: np.ndarray):
        """local: this rank's packed band buffer (u32).  Returns the frame on
        rank 0 (w*h u32), None elsewhere."""
        import torch
        from . import _lib
        local = np.ascontiguousarray(local, np.uint32)
        rect = np.ascontiguousarray(self.rect, np.int32)
        if self.rank != 0:
            n = self.part_pixels(self.rank)
            if n == 0:
                return None
            out = np.zeros(n, np.uint32)
            _lib.call("rt_pack_rect_host", self.w, self.h, self.world, self.rank, _lib.ptr(rect), _lib.ptr(local),
                      _lib.ptr(out))
            self.dist.send(torch.from_numpy(out.view(np.int32)), dst=0)
            return None
        sizes = [self.part_pixels(p) for p in range(1, self.world)]
        peers = np.zeros(max(1, sum(sizes)), np.uint32)
        off = 0
        for p, n in zip(range(1, self.world), sizes):
            if n > 0:
                buf = torch.zeros(n, dtype=torch.int32)
                self.dist.recv(buf, src=p)
                peers[off:off + n] = buf.numpy().view(np.uint32)
            off += n
        frame = np.zeros(self.w * self.h, np.uint32)
        _lib.call("rt_unpack_rect_host", self.w, self.h, self.world, _lib.ptr(rect), _lib.ptr(local),
                  _lib.ptr(peers), _lib.ptr(frame))
        return frame
