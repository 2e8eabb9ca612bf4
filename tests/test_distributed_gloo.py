"""World-size-2 gloo test of the frame gather (the N>1 path of bench.py) on CPU:
each rank packs its bands of an oracle-rendered frame, FrameGather collects
them on rank 0, which must reassemble the full frame exactly."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, collective, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cpp_cuda_raytracer_dev_amd.distributed import FrameGather, pack_bands_numpy
        from tests import helpers as H
        w, h = 200, 75
        argb, _, _ = H.oracle_render("rabbit_70k", w, h, 0)
        fg = FrameGather(dist, w, h, torch.device("cpu"), collective)
        fg.local.copy_(torch.from_numpy(pack_bands_numpy(argb, w, h, world, rank).view(np.int32)))
        fg.gather()
        if rank == 0:
            q.put(bool((fg.frame.numpy().view(np.uint32) == argb).all()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("collective", ["gather", "allgather"])
def test_frame_gather_world2(collective):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, collective, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
        assert p.exitcode == 0
    assert q.get(timeout=5) is True


# --------------------------------------------------------------------------
# The rectangle protocol of rt_comm_gather_frame (csrc/comm.cpp) across
# processes: every rank derives the rectangle alone (rt_frame_rect_host, from
# the host-side camera basis and root box), a peer sends exactly
# rt_rect_pixels(w, h, N, rank, rect) u32 to rank 0 in comm.cpp's order, and
# rank 0 assembles the frame with the background outside the rectangle
# (distributed.HostRectGather).  The assembled frame must be the oracle's
# (its committed full-frame hash).  No reference counterpart: the reference
# is single-GPU (TD/Trixel.cu:213); this is north_star's 1/2/4/8 split.

def _rect_geometry(name, w, h, coarse=8):
    from cpp_cuda_raytracer_dev_amd import raytracer as R
    from cpp_cuda_raytracer_dev_amd.distributed import frame_geometry
    from tests import helpers as H
    pos, la, up = (0.0, 0.1, -1.0), (0.0, 0.1, 0.0), (0.0, 1.0, 0.0)
    basis = R.camera_basis(w, h, R.film_w(w, h), np.float32(.024), np.float32(.055), pos, la, up)
    root = H.product_tree(name)[0]
    p = np.float32(pos)
    box = [np.float32(root["x0"]) - p[0], np.float32(root["x1"]) - p[0], np.float32(root["y0"]) - p[1],
           np.float32(root["y1"]) - p[1], np.float32(root["z0"]) - p[2], np.float32(root["z1"]) - p[2]]
    return frame_geometry(w, h, basis, box, bool(root["is_leaf"]), kernel=3, rays=0, coarse=coarse)


def _rect_worker(rank, world, port, name, w, h, coarse_of, q):
    import torch  # noqa: F401
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cpp_cuda_raytracer_dev_amd.distributed import HostRectGather, pack_bands_numpy
        from tests import helpers as H
        geom = _rect_geometry(name, w, h, coarse=coarse_of[rank])
        g = HostRectGather(dist, w, h, geom, None, 0)
        try:
            rect = g.verify()
        except RuntimeError as e:
            q.put((rank, "disagree", str(e)[:200]))
            return
        argb, _, _ = H.oracle_render(name, w, h, 0)
        frame = g.gather(pack_bands_numpy(argb, w, h, world, rank))
        sizes = [g.part_pixels(r) for r in range(world)]
        if rank == 0:
            import hashlib
            q.put((rank, "frame", rect, sizes, hashlib.sha256(frame.tobytes()).hexdigest(),
                   bool((frame == argb).all())))
        else:
            q.put((rank, "sent", rect, sizes))
    finally:
        dist.destroy_process_group()


def _run_rect(world, name, w, h, coarse_of):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rect_worker, args=(r, world, port, name, w, h, coarse_of, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    return sorted((q.get(timeout=10) for _ in range(world)), key=lambda t: t[0])


@pytest.mark.parametrize("world", [2, 4])
def test_rect_gather_protocol_gloo(world):
    from tests import helpers as H
    name, w, h = "rabbit_70k", 960, 540
    out = _run_rect(world, name, w, h, [8] * world)
    rects = {o[2] for o in out}
    assert len(rects) == 1, out  # every rank derived the same rectangle alone
    x0, x1, b0, b1 = rects.pop()
    assert 0 < x1 - x0 < w and 0 < b1 - b0 < (h + 7) // 8  # a real rectangle, not the whole frame
    sizes = out[0][3]
    assert all(o[3] == sizes for o in out)
    # each rank's part: its slots inside the rectangle, times its width
    for r in range(world):
        bands = [b for b in range(b0, b1) if b % world == r]
        assert sizes[r] == len(bands) * 8 * (x1 - x0)
    ent = H.frame_hashes()[f"{name}_{w}x{h}_m0"]
    assert out[0][1] == "frame" and out[0][5] is True
    assert out[0][4] == ent["argb_sha"]


def test_rect_gather_protocol_disagreement_raises():
    # rank 1 renders with other options (coarse groups per wave): verify must
    # raise on every rank before any transfer is posted
    out = _run_rect(2, "rabbit_70k", 320, 180, [8, 4])
    assert all(o[1] == "disagree" for o in out), out


def test_frame_rect_box_behind_eye_is_empty():
    """The box-behind-the-eye proof (rt_api.cpp box_behind, VERDICT r03 item
    5) from host-side inputs: the poses of bench.py --animate R+W.Q.T.W after
    the object has passed the camera give an empty gather rectangle (every
    pixel background, nothing sent) -- and the oracle renders those poses as
    background only; poses with the object in view keep a rectangle."""
    import bench
    from cpp_cuda_raytracer_dev_amd.distributed import frame_rect_host
    from oracle import motion as M
    from oracle import np_oracle as N
    from tests import helpers as H
    w, h = 320, 180
    g = _rect_geometry("dragon", w, h)
    masks = bench.key_masks("R+W.Q.T.W")
    cam = N.camera(w, h)
    ref = M.Motion(cam["pos"], cam["n"], cam["u"])
    seen = {"empty": 0, "kept": 0}
    for i in range(1501):
        ref.tick(masks[i % len(masks)])
        if i % 100 != 10:
            continue
        xf = np.asarray(ref.xform(), np.float32).reshape(12)
        rects = [frame_rect_host(g, xf, 0, n) for n in (1, 2, 4, 8)]
        _, ohit, _ = H.oracle_render("dragon", w, h, 0, xform=xf.reshape(3, 4))
        if rects[0] == (0, 0, 0, 0):
            assert all(r == (0, 0, 0, 0) for r in rects)
            assert not (ohit >= 0).any(), f"tick {i}: empty rectangle but the oracle shows the object"
            seen["empty"] += 1
        else:
            seen["kept"] += 1
            if (ohit >= 0).any():
                assert rects[0][1] > rects[0][0]
    assert seen["empty"] >= 5 and seen["kept"] >= 1, seen
