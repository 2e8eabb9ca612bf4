"""GPU parity: the HIP path against the oracle, bit-exact on the u32 frame and
the int64 hit buffer (BASELINE north_star: pixel-for-pixel).

Every comparison is exact (no tolerance): the HIP kernels evaluate the
reference's expressions in the same order and precision as the oracle.
"""
import numpy as np
import pytest

from cpp_cuda_raytracer_dev_amd import raytracer as R
from tests import helpers as H

pytestmark = pytest.mark.gpu


def _assert_same(a, b, what):
    argb, hit = a[0], a[1]
    oargb, ohit = b[0], b[1]
    bad_hit = np.flatnonzero(hit != ohit)
    bad_rgb = np.flatnonzero(argb != oargb)
    assert bad_hit.size == 0, f"{what}: {bad_hit.size} hit mismatches, first {bad_hit[:5]} {hit[bad_hit[:5]]} vs {ohit[bad_hit[:5]]}"
    assert bad_rgb.size == 0, f"{what}: {bad_rgb.size} colour mismatches, first {bad_rgb[:5]}"


def test_native_library_is_loaded():
    from cpp_cuda_raytracer_dev_amd import _lib
    L = _lib.lib()
    n = np.zeros(1, np.int32)
    import ctypes as C
    cnt = C.c_int()
    _lib.call("rt_device_count", C.byref(cnt))
    assert cnt.value >= 1
    assert L._name.endswith("librt_mi355x.so")


@pytest.mark.parametrize("name,w,h", [("dump_test", 64, 36), ("tester", 80, 45), ("dump", 48, 27)])
@pytest.mark.parametrize("mode", [0, 1])
def test_small_frames_vs_golden(name, w, h, mode):
    g = H.golden()
    s = H.GpuScene(name, w, h)
    argb, hit, _ = s.render(mode)
    key = f"{name}_{w}x{h}_m{mode}"
    _assert_same((argb, hit), (g[key + "_argb"], g[key + "_hit"]), key + " vs numpy golden")
    oargb, ohit, _ = H.oracle_render(name, w, h, mode)
    _assert_same((argb, hit), (oargb, ohit), key + " vs oracle")


KERNELS = [(2, 0, 0), (2, 2, 0), (2, 1, 0), (3, 2, 32), (3, 1, 32), (3, 0, 32), (3, 2, 16), (3, 2, 8), (3, 3, 16),
           (3, 3, 8), (3, 4, 16), (3, 5, 16), (3, 5, 8), (3, 3, 0), (3, 3, 32)]  # (KD kernel, tile order, rays/wave; 0 = automatic)


def _counters_match(cnt, ocnt, kernel):
    """Visit counters are order-independent and must match the oracle exactly;
    the accept-event count [2] is a DFS-order property, which the
    wave-cooperative kernel (3) replaces by the valid-candidate count (>=)."""
    got = [int(x) for x in cnt]
    want = [int(ocnt[i]) for i in (0, 1, 2, 3, 4)]
    if kernel == 3:
        assert got[2] >= want[2]
        got[2] = want[2]
    assert got == want


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("kernel,order,rays", KERNELS)
def test_tester_320x180(mode, kernel, order, rays):
    s = H.GpuScene("tester", 320, 180, kernel=kernel, tile_order=order, rays=rays)
    argb, hit, cnt = s.render(mode, count=True)
    oargb, ohit, ocnt = H.oracle_render("tester", 320, 180, mode)
    _assert_same((argb, hit), (oargb, ohit), f"tester m{mode}")
    if mode == 0:
        _counters_match(cnt, ocnt, kernel)


@pytest.mark.parametrize("kernel,order,rays", KERNELS)
def test_rabbit_960x540_kd_and_counters(kernel, order, rays):
    s = H.GpuScene("rabbit_70k", 960, 540, kernel=kernel, tile_order=order, rays=rays)
    argb, hit, cnt = s.render(0, count=True)
    oargb, ohit, ocnt = H.oracle_render("rabbit_70k", 960, 540, 0)
    _assert_same((argb, hit), (oargb, ohit), "rabbit kd")
    _counters_match(cnt, ocnt, kernel)
    g = H.golden()
    import hashlib
    assert hashlib.sha256(argb.tobytes()).hexdigest() == str(g["rabbit_70k_960x540_m0_argb_sha"])
    assert hashlib.sha256(hit.tobytes()).hexdigest() == str(g["rabbit_70k_960x540_m0_hit_sha"])


def test_rabbit_960x540_flat_band():
    s = H.GpuScene("rabbit_70k", 960, 540)
    argb, hit, _ = s.render(1)
    rows = (262, 278)  # a band through the rabbit against a live oracle render (the full frame: hash test below)
    oargb, ohit, _ = H.oracle_render("rabbit_70k", 960, 540, 1, rows=rows)
    sl = slice(rows[0] * 960, rows[1] * 960)
    assert (ohit[sl] >= 0).sum() > 100
    _assert_same((argb[sl], hit[sl]), (oargb[sl], ohit[sl]), "rabbit flat band")
    # the flat and KD results agree on this scene (no boundary-pruned hits here)
    kargb, khit, _ = s.render(0)
    assert (khit[sl] == hit[sl]).all()


def test_native_frame_loop_single_gpu():
    """rt_run_frames without a communicator: the timed frames equal the
    oracle's (committed hash), in one and in several buffer sets."""
    import hashlib
    import torch
    ent = H.frame_hashes()["dragon_960x540_m0"]
    s = H.GpuScene("dragon", 960, 540)
    st = torch.cuda.Stream()
    bufs = [torch.zeros(960 * 540, dtype=torch.int32, device="cuda:0") for _ in range(3)]
    for n in (1, 3):
        loop = R.FrameLoop(s.cam, bufs[:n], render_stream=st.cuda_stream, event_every=4)
        ms, cnt, host = loop.run(10)
        assert cnt == 3 and ms > 0
        for b in bufs[:n]:
            a = b.cpu().numpy().view(np.uint32)
            if H.mesh_matches(ent):
                assert hashlib.sha256(a.tobytes()).hexdigest() == ent["argb_sha"]
    assert s.cam.device_error() == 0


@pytest.mark.parametrize("inflight,nbuf", [(2, 2), (2, 4), (3, 3), (4, 4)])
def test_native_frame_loop_inflight(inflight, nbuf):
    """Frames in flight on the camera's render lanes: every buffer holds the
    oracle's frame (committed hash) after enough frames for the tile-cost
    samples and cost-order uploads to run while other lanes render."""
    import hashlib
    import torch
    from cpp_cuda_raytracer_dev_amd import _lib
    ent = H.frame_hashes()["dragon_960x540_m0"]
    s = H.GpuScene("dragon", 960, 540)
    st = torch.cuda.Stream()
    bufs = [torch.full((960 * 540,), 0x7BADBEEF, dtype=torch.int32, device="cuda:0") for _ in range(nbuf)]
    torch.cuda.synchronize()
    loop = R.FrameLoop(s.cam, bufs, render_stream=st.cuda_stream, event_every=5, inflight=inflight)
    ms, cnt, host = loop.run(80)
    assert cnt == 16 and ms > 0
    for b in bufs:
        a = b.cpu().numpy().view(np.uint32)
        if H.mesh_matches(ent):
            assert hashlib.sha256(a.tobytes()).hexdigest() == ent["argb_sha"]
        else:
            assert (a == bufs[0].cpu().numpy().view(np.uint32)).all()
    assert s.cam.device_error() == 0
    if nbuf == 2 and inflight == 2:
        with pytest.raises(_lib.RtError):  # sets must split evenly over the lanes
            R.FrameLoop(s.cam, bufs[:1] * 3, render_stream=st.cuda_stream, inflight=2).run(1)


@pytest.mark.parametrize("inflight", [1, 2])
def test_native_frame_loop_poses(inflight):
    """rt_frame_loop.xforms: frame k renders pose k mod n (a moving object's
    per-frame transforms), with one or two frames in flight; each buffer set
    holds the frame of its pose, equal to a single render at that pose."""
    import torch
    w, h = 320, 180
    s = H.GpuScene("rabbit_70k", w, h)
    poses = [_rot_y(0.0), _rot_y(7.0), _rot_y(-5.0, (0.004, 0.0, 0.0)), _rot_y(11.0, (0.0, 0.003, 0.0))]
    fulls = [s.render(0, xform=xf)[0] for xf in poses]
    st = torch.cuda.Stream()
    bufs = [torch.full((w * h,), 0x7BADBEEF, dtype=torch.int32, device="cuda:0") for _ in poses]
    torch.cuda.synchronize()
    loop = R.FrameLoop(s.cam, bufs, render_stream=st.cuda_stream, event_every=3, inflight=inflight, xforms=poses)
    loop.run(10)
    for k, (b, f) in enumerate(zip(bufs, fulls)):
        assert (b.cpu().numpy().view(np.uint32) == f).all(), f"pose {k}"
    assert s.cam.device_error() == 0


def test_auto_rays_choice():
    """RT_OPT_RAYS 0 (default): 8 pixels per wave when this rank's share of
    the object's screen rectangle holds fewer than 2,048 16-ray units (a rank
    of 2 at 960x540: 1.7k), else 16 (960x540 whole: 3.4k; 1080p: 13.4k)."""
    import torch
    from cpp_cuda_raytracer_dev_amd import _lib
    for (w, h), n, want in (((960, 540), 1, 16), ((1920, 1080), 1, 16), ((960, 540), 2, 8), ((1920, 1080), 8, 8)):
        s = H.GpuScene("dragon", w, h)
        buf = torch.zeros(R.packed_pixels(w, h, n), dtype=torch.int32, device="cuda:0")
        s.cam.render_into(buf, tile=(n, 0))
        torch.cuda.synchronize()
        assert s.cam.get_option(_lib.RT_OPT_RAYS_USED) == want, (w, h, n)


@pytest.mark.parametrize("shadow", [False, True])
def test_tall_tree_stays_on_kernel3(shadow):
    """A 3.1M-triangle stand-in has a 22-level tree (the former path-code
    limit of kernel 3 was 21): it renders in kernel 3, shadows included, and
    its rows through the object equal the oracle's (the full frame: the hash
    test).  The oracle walks the product's tree here, which tests/test_host_cpu.py
    proves equal to the literal create_kd restatement."""
    from cpp_cuda_raytracer_dev_amd import _lib
    import ctypes as C
    s = H.GpuScene("big", 1920, 1080, kernel=3)
    depth = C.c_int32()
    _lib.call("rt_camera_info", s.cam._h, None, None, C.byref(depth))
    assert depth.value == 22
    argb, hit, _ = s.render(0, shadow=shadow)
    assert s.cam.get_option(_lib.RT_OPT_KERNEL) == 3
    pts = H.mesh("big")[0]
    from oracle import _oracle as O
    pn = H.product_tree("big")
    on = np.zeros(len(pn), O.NODE_DTYPE)
    for k in pn.dtype.names:
        on[k] = pn[k]
    rows = (520, 560)
    osc = O.Scene(pts, O.default_rad(len(pts)), on, O.camera(1920, 1080))
    oargb, ohit, _ = osc.render(0, rows=rows, nthreads=H.ORACLE_THREADS, shadow=shadow)
    osc.close()
    sl = slice(rows[0] * 1920, rows[1] * 1920)
    assert (ohit[sl] >= 0).sum() > 1000
    _assert_same((argb[sl], hit[sl]), (oargb[sl], ohit[sl]), f"big 22-level tree shadow={shadow}")


@pytest.mark.parametrize("order,height", [(0, 3), (1, 3), (2, 2), (2, 3), (2, 5)])
@pytest.mark.parametrize("kernel", [2, 3])
@pytest.mark.parametrize("shadow", [False, True])
def test_interior_record_orders(order, height, kernel, shadow):
    """The interior records' order (BFS, DFS preorder, treelets) is internal:
    every kernel renders the oracle's frame and counters with each."""
    from cpp_cuda_raytracer_dev_amd import _lib
    if shadow and kernel != 3:
        pytest.skip("shadow rays run in kernel 3")
    s = H.GpuScene("dragon", 960, 540, kernel=kernel)
    s.trixel.set_option(_lib.RT_SCENE_TREELET_HEIGHT, height)
    s.trixel.set_option(_lib.RT_SCENE_ORDER, order)
    assert s.trixel.get_option(_lib.RT_SCENE_ORDER) == order
    argb, hit, cnt = s.render(0, count=True, shadow=shadow)
    oargb, ohit, ocnt = H.oracle_render("dragon", 960, 540, 0, shadow=shadow)
    _assert_same((argb, hit), (oargb, ohit), f"order {order}/{height} kernel {kernel}")
    _counters_match(cnt, ocnt, kernel)


@pytest.mark.parametrize("variant", [9, 12])
@pytest.mark.parametrize("name,w,h", [("dump_test", 64, 36), ("tester", 80, 45), ("dump", 48, 27),
                                      ("tester", 33, 9)])
def test_flat_kernel_variants(variant, name, w, h):
    """Both forms of the flat-list kernel (one pass, and the list in 16
    chunks; dump_test has an odd count: a dead twin) render the oracle's
    frame, counters included; every other form is refused."""
    from cpp_cuda_raytracer_dev_amd import _lib
    s = H.GpuScene(name, w, h)
    s.cam.set_option(_lib.RT_OPT_FLAT, variant)
    argb, hit, cnt = s.render(1, count=True)
    oargb, ohit, ocnt = H.oracle_render(name, w, h, 1)
    _assert_same((argb, hit), (oargb, ohit), f"{name} flat v{variant}")
    assert [int(cnt[i]) for i in (1, 2, 3)] == [int(ocnt[i]) for i in (1, 2, 3)]
    argb, hit, _ = s.render(1)
    _assert_same((argb, hit), (oargb, ohit), f"{name} flat v{variant} timed")
    for bad in (0, 5, 10, 13):
        with pytest.raises(_lib.RtError):
            s.cam.set_option(_lib.RT_OPT_FLAT, bad)


@pytest.mark.parametrize("variant", [9, 12])
def test_flat_kernel_variants_rabbit_hash(variant):
    import hashlib
    from cpp_cuda_raytracer_dev_amd import _lib
    ent = H.frame_hashes()["rabbit_70k_960x540_m1"]
    s = H.GpuScene("rabbit_70k", 960, 540)
    s.cam.set_option(_lib.RT_OPT_FLAT, variant)
    argb, hit, cnt = s.render(1, count=True)
    assert hashlib.sha256(argb.tobytes()).hexdigest() == ent["argb_sha"]
    assert hashlib.sha256(hit.tobytes()).hexdigest() == ent["hit_sha"]
    assert [int(cnt[i]) for i in (1, 2, 3)] == [ent["counters"][i] for i in (1, 2, 3)]
    # the timed (non-counting) instance as well
    argb, hit, _ = s.render(1)
    assert hashlib.sha256(argb.tobytes()).hexdigest() == ent["argb_sha"]
    assert hashlib.sha256(hit.tobytes()).hexdigest() == ent["hit_sha"]


@pytest.mark.parametrize("variant", [9, 12])
@pytest.mark.parametrize("ntri", [1, 2, 3, 257])
def test_flat_signed_layout_edge_triangles(variant, ntri):
    """The signed pair layout on triangles of both windings, facing
    and behind the camera, zero-area ones and ones whose plane holds the camera
    (d_w = 0): every form renders the oracle's flat frame and counters."""
    import numpy as np
    from cpp_cuda_raytracer_dev_amd import _lib
    from oracle import _oracle as O
    rng = np.random.default_rng(1000 + ntri)
    v = rng.uniform(-0.4, 0.4, size=(3 * ntri, 3)).astype(np.float32)
    v[:, 1] += 0.1
    f = np.arange(3 * ntri, dtype=np.int32).reshape(ntri, 3)
    if ntri > 3:
        f[1::2] = f[1::2, ::-1]                        # both windings
        v[3 * 5 + 2] = v[3 * 5]                        # zero-area triangle (e2 = 0)
        v[3 * 7:3 * 7 + 3, 0] = 0.0                    # plane x = 0 holds the camera: d_w = 0
        v[3 * 9:3 * 9 + 3, 2] -= 1.5                   # behind the camera
    pts, _, leafs = R.assemble_mesh(v, f)
    opts, _ = O.assemble(v, np.full(ntri, 3, np.int32), f.reshape(-1))
    assert pts.tobytes() == opts.tobytes()
    w, h = 40, 24
    trixel = R.Trixel(len(pts), pts)
    cam = R.Camera.default(w, h)
    cam.set_option(_lib.RT_OPT_FLAT, variant)
    obj = R.Object(trixel)
    cam.add_object(obj)
    obj.render(cam, mode=1, flags=R.RT_FLAG_WRITE_HIT | R.RT_FLAG_COUNT)
    cam.color_pixels(R.PHONG_COLOR_TAG)
    cnt = cam.counters()
    ocam = O.camera(w, h)
    osc = O.Scene(pts, O.default_rad(len(pts)), None, ocam)
    try:
        oargb, ohit, ocnt = osc.render(1, nthreads=4)
    finally:
        osc.close()
    _assert_same((cam.h_color.copy(), cam.h_rmi.copy()), (oargb, ohit), f"signed flat v{variant} n{ntri}")
    assert [int(cnt[i]) for i in (1, 2, 3)] == [int(ocnt[i]) for i in (1, 2, 3)]
    obj.render(cam, mode=1, flags=R.RT_FLAG_WRITE_HIT)  # the timed (non-counting) instance
    cam.color_pixels(R.PHONG_COLOR_TAG)
    _assert_same((cam.h_color.copy(), cam.h_rmi.copy()), (oargb, ohit), f"signed flat v{variant} n{ntri} timed")


# Full frames against the oracle's committed SHA-256 (tests/golden/frame_hashes.json,
# tests/golden/make_hashes.py): every BASELINE config at its full size (C2's
# flat rabbit 960x540 = 3.6e10 ray-triangle tests, C5's happy 3840x2160 with
# shadow rays), the bench's headline frame and the >= 90 % coverage views.
@pytest.mark.parametrize("key", H.hash_keys())
def test_full_frame_vs_oracle_hash(key):
    import hashlib
    ent = H.frame_hashes()[key]
    s = H.GpuScene(ent["scene"], ent["w"], ent["h"], cam_kw=H.view_kw(ent))
    argb, hit, cnt = s.render(ent["mode"], shadow=ent["shadow"], count=ent["mode"] == 0)
    if not H.mesh_matches(ent):
        # this host's numpy built other stand-in vertex bits: the live oracle decides
        oargb, ohit, ocnt = H.oracle_render(ent["scene"], ent["w"], ent["h"], ent["mode"], cam_kw=H.view_kw(ent),
                                            shadow=ent["shadow"])
        _assert_same((argb, hit), (oargb, ohit), key + " vs oracle (stand-in mesh differs from the hashed one)")
        return
    assert hashlib.sha256(argb.tobytes()).hexdigest() == ent["argb_sha"], f"{key}: u32 frame differs from the oracle"
    assert hashlib.sha256(hit.tobytes()).hexdigest() == ent["hit_sha"], f"{key}: hit buffer differs from the oracle"
    assert int((hit >= 0).sum()) == ent["hit_pixels"]
    if ent["mode"] == 0:
        _counters_match(cnt, ent["counters"], 3)


@pytest.mark.parametrize("key,rays", [("dragon_960x540_m0", 0), ("knot_960x540_m0", 0), ("knot_960x540_m0", 16),
                                      ("dragon_960x540_m0_shadow", 0), ("dragon_960x540_m0", 8),
                                      ("knot_960x540_m0", 8), ("dragon_960x540_m0_shadow", 8),
                                      ("dragon_1920x1080_m0", 0), ("knot_1920x1080_m0", 0)])
def test_split_tiles_same_frame(key, rays):
    """Tile order 3 splits the heaviest 16-ray tiles into two 8-ray halves
    (8-ray units: two 4-pixel halves) once a cost sample has arrived
    (RT_OPT_SPLIT_USED > 0; above half the heaviest tile's cost in grids of
    fewer than 2,048 tiles, above 75 % in larger ones): the frame and hit
    buffer stay the oracle's (committed hashes)."""
    import hashlib
    import torch
    from cpp_cuda_raytracer_dev_amd import _lib
    if key.endswith("_shadow"):  # no committed hash: the oracle renders it here
        w, h = 960, 540
        oargb, ohit = H.oracle_render("dragon", w, h, 0, shadow=True)[:2]
        ent = {"scene": "dragon", "shadow": True, "argb_sha": hashlib.sha256(oargb.tobytes()).hexdigest(),
               "hit_sha": hashlib.sha256(np.ascontiguousarray(ohit).tobytes()).hexdigest()}
    else:
        ent = H.frame_hashes()[key]
        if not H.mesh_matches(ent):
            pytest.skip("stand-in mesh bits differ on this host")
        w, h = ent["w"], ent["h"]
    s = H.GpuScene(ent["scene"], w, h, rays=rays)
    dev = torch.device("cuda:0")
    out = torch.zeros(w * h, dtype=torch.int32, device=dev)
    hit = torch.zeros(w * h, dtype=torch.int64, device=dev)
    flags = R.RT_FLAG_WRITE_HIT | (R.RT_FLAG_SHADOW if ent["shadow"] else 0)
    # cost samples are read back by event queries, never waits: when the host
    # enqueues faster than the GPU renders, a sample may not have arrived
    # after a burst of frames, so render in bursts with a sync between them
    for _ in range(16):
        for _ in range(16):
            s.cam.render_into(out, hit, flags=flags)
        torch.cuda.synchronize()
        if s.cam.get_option(_lib.RT_OPT_SPLIT_USED) > 0:
            break
    assert s.cam.get_option(_lib.RT_OPT_RAYS_USED) == (rays or 16)
    assert s.cam.get_option(_lib.RT_OPT_SPLIT_USED) > 0
    s.cam.render_into(out, hit, flags=flags)
    torch.cuda.synchronize()
    argb = out.cpu().numpy().view(np.uint32)
    assert hashlib.sha256(argb.tobytes()).hexdigest() == ent["argb_sha"], key
    assert hashlib.sha256(hit.cpu().numpy().tobytes()).hexdigest() == ent["hit_sha"], key
    assert s.cam.device_error(reset=True) == 0


@pytest.mark.parametrize("w,h", [(960, 540), (1920, 1080)])
@pytest.mark.parametrize("kernel,order,rays", KERNELS)
def test_dragon_standin_kd(w, h, kernel, order, rays):
    s = H.GpuScene("dragon", w, h, kernel=kernel, tile_order=order, rays=rays)
    argb, hit, cnt = s.render(0, count=True)
    oargb, ohit, ocnt = H.oracle_render("dragon", w, h, 0)
    _assert_same((argb, hit), (oargb, ohit), f"dragon {w}x{h}")
    _counters_match(cnt, ocnt, kernel)
    assert (hit >= 0).mean() > 0.02


def test_happy_standin_kd_2160p_rows():
    # 4K frame on the GPU; oracle on a band of rows (full 4K oracle is minutes of CPU)
    w, h = 3840, 2160
    s = H.GpuScene("happy", w, h)
    argb, hit, _ = s.render(0)
    rows = (1000, 1100)
    oargb, ohit, _ = H.oracle_render("happy", w, h, 0, rows=rows)
    sl = slice(rows[0] * w, rows[1] * w)
    assert (ohit[sl] >= 0).sum() > 1000
    _assert_same((argb[sl], hit[sl]), (oargb[sl], ohit[sl]), "happy 4K band")


def _rot_y(deg, t=(0.0, 0.0, 0.0)):
    a = np.deg2rad(deg)
    c, s = np.float32(np.cos(a)), np.float32(np.sin(a))
    return np.array([[c, 0, s, t[0]], [0, 1, 0, t[1]], [-s, 0, c, t[2]]], np.float32).reshape(12)


@pytest.mark.parametrize("xf", [_rot_y(0.0, (0.01, -0.005, 0.02)), _rot_y(17.0), _rot_y(-9.0, (0.0, 0.01, 0.0))])
@pytest.mark.parametrize("kernel", [2, 3])
def test_object_transform(xf, kernel):
    """Non-identity rot_m exercises the ray rotation, obj_d offsets and normal rotation of TD/Trixel.cu:60-140."""
    s = H.GpuScene("rabbit_70k", 320, 180, kernel=kernel)
    argb, hit, _ = s.render(0, xform=xf)
    oargb, ohit, _ = H.oracle_render("rabbit_70k", 320, 180, 0, xform=xf)
    assert (ohit >= 0).sum() > 100
    _assert_same((argb, hit), (oargb, ohit), "xform")


def _poses(n, seed=7):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        pos = (np.array([-0.02, 0.11, 0.0]) + (0.35 + 0.4 * rng.random()) * d).astype(np.float32)
        out.append(dict(pos=tuple(float(x) for x in pos), look_at=(-0.02, 0.11, 0.0)))
    return out


@pytest.mark.parametrize("pose", _poses(6))
def test_camera_poses_rabbit(pose):
    s = H.GpuScene("rabbit_70k", 240, 135, cam_kw=pose)
    argb, hit, _ = s.render(0)
    oargb, ohit, _ = H.oracle_render("rabbit_70k", 240, 135, 0, cam_kw=pose)
    _assert_same((argb, hit), (oargb, ohit), f"pose {pose}")


def _model_poses(name, n=16, seed=7):
    """SURVEY.md §8d's parity fuzz: n seeded camera poses on a sphere around
    the model's box centre, 1.5-3.5 box diagonals away, looking at it."""
    pts = np.asarray(H.mesh(name)[0], np.float32).reshape(-1, 3)
    lo, hi = pts.min(axis=0), pts.max(axis=0)
    c, diag = (lo + hi) / 2, float(np.linalg.norm(hi - lo))
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        pos = (c + (1.5 + 2.0 * rng.random()) * diag * d).astype(np.float32)
        out.append(dict(pos=tuple(float(x) for x in pos), look_at=tuple(float(x) for x in c)))
    return out


@pytest.mark.parametrize("name", ["dragon", "happy", "knot", "rabbit_70k"])
def test_camera_pose_fuzz(name):
    """16 seeded poses around each model, kernel 3 defaults
    (two-level iterations, cost order, auto rays): frames and hit indices
    equal the oracle's at every pose."""
    for k, pose in enumerate(_model_poses(name)):
        s = H.GpuScene(name, 160, 90, cam_kw=pose)
        argb, hit, _ = s.render(0)
        argb2, hit2, _ = s.render(0)  # a second frame: the cost order of the first applies
        oargb, ohit, _ = H.oracle_render(name, 160, 90, 0, cam_kw=pose)
        _assert_same((argb, hit), (oargb, ohit), f"{name} pose {k} {pose}")
        _assert_same((argb2, hit2), (oargb, ohit), f"{name} pose {k} second frame")
        assert s.cam.device_error(reset=True) == 0


@pytest.mark.parametrize("items", [1, 2, 96])
@pytest.mark.parametrize("rays", [32, 16, 8])
@pytest.mark.parametrize("shadow", [False, True])
def test_items_per_lane(items, rays, shadow):
    """Kernel 3 pops one or two items per lane per iteration (96: two only from
    96 pooled items on); same frame and counters."""
    s = H.GpuScene("dragon", 960, 540, kernel=3, rays=rays, items=items)
    argb, hit, cnt = s.render(0, count=True, shadow=shadow)
    oargb, ohit, ocnt = H.oracle_render("dragon", 960, 540, 0, shadow=shadow)
    _assert_same((argb, hit), (oargb, ohit), f"items {items} rays {rays}")
    _counters_match(cnt, ocnt, 3)


@pytest.mark.parametrize("cap", [89, 96, 200])
def test_pool_capacity_fallback(cap):
    """A small item pool forces the wave-cooperative kernel's single-item
    (DFS-like) pops; the frame must not change."""
    from cpp_cuda_raytracer_dev_amd import _lib
    s = H.GpuScene("dragon", 960, 540, kernel=3)
    s.cam.set_option(_lib.RT_OPT_POOL_CAP, cap)
    argb, hit, cnt = s.render(0, count=True)
    oargb, ohit, ocnt = H.oracle_render("dragon", 960, 540, 0)
    _assert_same((argb, hit), (oargb, ohit), f"pool cap {cap}")
    _counters_match(cnt, ocnt, 3)


def test_two_level_depth_option():
    """The scene's two-level depth: floor(log2 n) - 2 in BFS record order (the
    top levels of the reference's tree are full), none in DFS order, the top
    treelet's in treelet order; read only."""
    from cpp_cuda_raytracer_dev_amd import _lib
    for name in ("dragon", "rabbit_70k", "tester"):
        s = H.GpuScene(name, 64, 36)
        n = len(H.mesh(name)[0])
        t = s.trixel
        assert t.get_option(_lib.RT_SCENE_TWO_LEVEL_DEPTH) == int(np.floor(np.log2(n))) - 2, name
        t.set_option(_lib.RT_SCENE_ORDER, 1)
        assert t.get_option(_lib.RT_SCENE_TWO_LEVEL_DEPTH) == -1, name
        t.set_option(_lib.RT_SCENE_TREELET_HEIGHT, 4)
        t.set_option(_lib.RT_SCENE_ORDER, 2)
        assert t.get_option(_lib.RT_SCENE_TWO_LEVEL_DEPTH) == min(2, int(np.floor(np.log2(n))) - 2), name
        t.set_option(_lib.RT_SCENE_ORDER, 0)
        with pytest.raises(Exception):
            t.set_option(_lib.RT_SCENE_TWO_LEVEL_DEPTH, 3)


@pytest.mark.parametrize("name,w,h", [("dragon", 960, 540), ("knot", 480, 270), ("rabbit_70k", 320, 180)])
@pytest.mark.parametrize("rays", [16, 8])
@pytest.mark.parametrize("shadow", [False, True])
@pytest.mark.parametrize("two_level", [True, False])
def test_two_level_iterations(name, w, h, rays, shadow, two_level):
    """Kernel 3's two-level iterations (pools of at most 16 items: a quad of
    lanes per item, the children's records in the same round trip) and the
    one-level walk (debug bit 1024) render the oracle's frame with its
    counters."""
    from cpp_cuda_raytracer_dev_amd import _lib
    s = H.GpuScene(name, w, h, kernel=3, rays=rays)
    if not two_level:
        s.cam.set_option(_lib.RT_OPT_DEBUG, 1024)
    argb, hit, cnt = s.render(0, count=True, shadow=shadow)
    oargb, ohit, ocnt = H.oracle_render(name, w, h, 0, shadow=shadow)
    _assert_same((argb, hit), (oargb, ohit), f"{name} two-level {two_level}")
    _counters_match(cnt, ocnt, 3)
    argb2, hit2, _ = s.render(0, shadow=shadow)
    _assert_same((argb2, hit2), (oargb, ohit), f"{name} two-level {two_level} (timed instance)")
    assert s.cam.device_error(reset=True) == 0


@pytest.mark.parametrize("w,h", [(81, 45), (1, 1), (33, 9), (7, 130)])
@pytest.mark.parametrize("kernel,order,rays", KERNELS)
def test_odd_resolutions(w, h, kernel, order, rays):
    for mode in (0, 1):
        s = H.GpuScene("tester", w, h, kernel=kernel, tile_order=order, rays=rays)
        argb, hit, _ = s.render(mode)
        oargb, ohit, _ = H.oracle_render("tester", w, h, mode)
        _assert_same((argb, hit), (oargb, ohit), f"tester {w}x{h} m{mode}")


@pytest.mark.parametrize("nranks", [2, 3, 8])
@pytest.mark.parametrize("kernel,order,rays", KERNELS)
def test_band_tiles_unpack(nranks, kernel, order, rays):
    import torch
    from cpp_cuda_raytracer_dev_amd import raytracer as R
    w, h = 1920, 1080
    s = H.GpuScene("dragon", w, h, kernel=kernel, tile_order=order, rays=rays)
    full, fhit, _ = s.render(0)
    npk = R.packed_pixels(w, h, nranks)
    dev = torch.device("cuda:0")
    gathered = torch.zeros(nranks * npk, dtype=torch.int32, device=dev)
    for r in range(nranks):
        s.cam.render_into(gathered[r * npk:(r + 1) * npk], mode=0, tile=(nranks, r))
    frame = torch.zeros(w * h, dtype=torch.int32, device=dev)
    R.unpack_bands(0, w, h, nranks, gathered, frame)
    torch.cuda.synchronize()
    got = frame.cpu().numpy().view(np.uint32)
    assert (got == full).all()
    from cpp_cuda_raytracer_dev_amd import distributed as D
    ref = D.unpack_bands_numpy(gathered.cpu().numpy().view(np.uint32), w, h, nranks)
    assert (ref == full).all()


def test_render_into_stream_and_repeat():
    """Repeated frames on a non-default stream are identical (stateless frames)."""
    import torch
    s = H.GpuScene("dragon", 960, 540)
    ref, _, _ = s.render(0)
    st = torch.cuda.Stream()
    out = torch.zeros(960 * 540, dtype=torch.int32, device="cuda:0")
    with torch.cuda.stream(st):
        for _ in range(5):
            s.cam.render_into(out, mode=0, stream=st.cuda_stream)
    st.synchronize()
    assert (out.cpu().numpy().view(np.uint32) == ref).all()


# ------------------------------------------------------------- shadow rays
# RT_FLAG_SHADOW (config C5): the wave-cooperative kernel's
# second pool walk against the oracle's trace_shadow.  The any-hit result does
# not depend on visit order, so frames are bit-exact; with counters on, the
# shadow walks visit every node the oracle visits (no early exit).
SHADOW_KERNELS = [(3, 1, 32), (3, 2, 32), (3, 2, 16), (3, 2, 8)]


@pytest.mark.parametrize("name,w,h", [("rabbit_70k", 960, 540), ("dragon", 960, 540)])
@pytest.mark.parametrize("kernel,order,rays", SHADOW_KERNELS)
def test_shadow_kd(name, w, h, kernel, order, rays):
    s = H.GpuScene(name, w, h, kernel=kernel, tile_order=order, rays=rays)
    argb, hit, cnt = s.render(0, count=True, shadow=True)
    oargb, ohit, ocnt = H.oracle_render(name, w, h, 0, shadow=True)
    _assert_same((argb, hit), (oargb, ohit), f"{name} shadow")
    _counters_match(cnt, ocnt, 3)
    assert ((argb == 0) & (hit >= 0)).sum() > 100
    # without counters the shadow walk stops early; the frame is the same
    argb2, hit2, _ = s.render(0, shadow=True)
    _assert_same((argb2, hit2), (oargb, ohit), f"{name} shadow (early exit)")


def test_shadow_golden_hash():
    import hashlib
    g = H.golden()
    s = H.GpuScene("rabbit_70k", 960, 540)
    argb, _, cnt = s.render(0, count=True, shadow=True)
    assert hashlib.sha256(argb.tobytes()).hexdigest() == str(g["rabbit_70k_960x540_shadow_argb_sha"])
    _counters_match(cnt, g["rabbit_70k_960x540_shadow_counters"], 3)


def test_shadow_dragon_1080p():
    s = H.GpuScene("dragon", 1920, 1080)
    argb, hit, cnt = s.render(0, count=True, shadow=True)
    oargb, ohit, ocnt = H.oracle_render("dragon", 1920, 1080, 0, shadow=True)
    _assert_same((argb, hit), (oargb, ohit), "dragon 1080p shadow")
    _counters_match(cnt, ocnt, 3)


def test_shadow_happy_2160p_rows():
    """Config C5 (happy stand-in, 3840x2160, one shadow ray per hit) on a band of rows."""
    w, h = 3840, 2160
    s = H.GpuScene("happy", w, h)
    argb, hit, _ = s.render(0, shadow=True)
    rows = (900, 1000)
    oargb, ohit, _ = H.oracle_render("happy", w, h, 0, rows=rows, shadow=True)
    sl = slice(rows[0] * w, rows[1] * w)
    assert ((oargb[sl] == 0) & (ohit[sl] >= 0)).sum() > 1000
    _assert_same((argb[sl], hit[sl]), (oargb[sl], ohit[sl]), "happy 4K shadow band")


@pytest.mark.parametrize("xf", [_rot_y(0.0, (0.01, -0.005, 0.02)), _rot_y(17.0)])
def test_shadow_object_transform(xf):
    s = H.GpuScene("rabbit_70k", 320, 180, kernel=3)
    argb, hit, _ = s.render(0, xform=xf, shadow=True)
    oargb, ohit, _ = H.oracle_render("rabbit_70k", 320, 180, 0, xform=xf, shadow=True)
    _assert_same((argb, hit), (oargb, ohit), "shadow xform")


@pytest.mark.parametrize("cap", [89, 200])
def test_shadow_pool_capacity_fallback(cap):
    from cpp_cuda_raytracer_dev_amd import _lib
    s = H.GpuScene("dragon", 960, 540, kernel=3)
    s.cam.set_option(_lib.RT_OPT_POOL_CAP, cap)
    argb, hit, cnt = s.render(0, count=True, shadow=True)
    oargb, ohit, ocnt = H.oracle_render("dragon", 960, 540, 0, shadow=True)
    _assert_same((argb, hit), (oargb, ohit), f"shadow pool cap {cap}")
    _counters_match(cnt, ocnt, 3)


def test_shadow_band_tiles():
    import torch
    from cpp_cuda_raytracer_dev_amd import raytracer as R
    w, h, nranks = 960, 540, 3
    s = H.GpuScene("dragon", w, h)
    full, _, _ = s.render(0, shadow=True)
    npk = R.packed_pixels(w, h, nranks)
    gathered = torch.zeros(nranks * npk, dtype=torch.int32, device="cuda:0")
    for r in range(nranks):
        s.cam.render_into(gathered[r * npk:(r + 1) * npk], mode=0, flags=R.RT_FLAG_SHADOW, tile=(nranks, r))
    frame = torch.zeros(w * h, dtype=torch.int32, device="cuda:0")
    R.unpack_bands(0, w, h, nranks, gathered, frame)
    torch.cuda.synchronize()
    assert (frame.cpu().numpy().view(np.uint32) == full).all()


@pytest.mark.parametrize("kernel,mode", [(2, 0), (3, 1)])
def test_shadow_rejected_outside_kernel3_kd(kernel, mode):
    from cpp_cuda_raytracer_dev_amd import _lib
    s = H.GpuScene("tester", 64, 36, kernel=kernel)
    with pytest.raises(_lib.RtError):
        s.render(mode, shadow=True)


# ------------------------------------------------------- coarse background
# Kernel 3 splits a frame into fine tiles (the root box's screen rectangle,
# one unit per wave) and coarse 8x8 groups elsewhere (k_coarse_kd3, several
# per wave), which run the same root test and trace any sub-tile where a ray
# passes.  Frames and counters must not depend on the split: coarse off (0),
# one or many groups per wave, and the diagnostic "every group coarse" (debug
# bit 4), which sends the whole object through the coarse kernel's tracing;
# debug bit 8 runs the coarse kernel on a side stream beside the fine one.
# The coarse kernel first tries its certain-miss test (hardware rsqrt/rcp
# with a 1e-3 margin; under a transform, root_certain_miss_xf with explicit
# error bounds); any doubt takes the exact test.
COARSE = [(0, None), (1, None), (8, None), (32, None), (8, 4), (1, 4), (32, 4), (8, 8), (2, 12)]  # (groups per wave, debug)


@pytest.mark.parametrize("coarse,debug", COARSE)
@pytest.mark.parametrize("rays", [32, 16, 8])
@pytest.mark.parametrize("name,w,h", [("rabbit_70k", 320, 180), ("dragon", 960, 540), ("tester", 81, 45)])
def test_coarse_split(name, w, h, rays, coarse, debug):
    s = H.GpuScene(name, w, h, kernel=3, rays=rays, coarse=coarse, debug=debug)
    argb, hit, cnt = s.render(0, count=True)
    oargb, ohit, ocnt = H.oracle_render(name, w, h, 0)
    _assert_same((argb, hit), (oargb, ohit), f"{name} coarse {coarse} debug {debug}")
    _counters_match(cnt, ocnt, 3)
    argb2, hit2, _ = s.render(0)
    _assert_same((argb2, hit2), (oargb, ohit), f"{name} coarse {coarse} debug {debug} (no counters)")


@pytest.mark.parametrize("debug", [None, 4])
@pytest.mark.parametrize("pose", _poses(6, seed=11))
def test_coarse_poses_and_transforms(pose, debug):
    for xf in (None, _rot_y(23.0, (0.02, 0.0, -0.01))):
        s = H.GpuScene("rabbit_70k", 200, 120, cam_kw=pose, kernel=3, debug=debug)
        argb, hit, _ = s.render(0, xform=xf)
        oargb, ohit, _ = H.oracle_render("rabbit_70k", 200, 120, 0, cam_kw=pose, xform=xf)
        _assert_same((argb, hit), (oargb, ohit), f"pose {pose} xf {xf is not None} debug {debug}")


def _quat_xform(axis, deg, t):
    """rot_m rows of a rotation by `deg` about `axis` (float32) and offset t."""
    a = np.asarray(axis, np.float64)
    a = a / np.linalg.norm(a)
    h = np.deg2rad(deg) / 2
    w, x, y, z = np.cos(h), *(np.sin(h) * a)
    m = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                  [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                  [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
    return np.hstack([m, np.asarray(t, np.float64).reshape(3, 1)]).astype(np.float32).reshape(12)


# general rotations (random axes, up to 120 degrees), offsets, and a signed
# permutation (exact zeros in rot_m, so rotated components vanish with the
# camera's own) exercise root_certain_miss_xf's bounds against the oracle
_XF_RNG = np.random.default_rng(20261017)
_GENERAL_XFS = [_quat_xform(_XF_RNG.normal(size=3), _XF_RNG.uniform(-120, 120), _XF_RNG.uniform(-0.03, 0.03, 3))
                for _ in range(5)] + [np.array([0, 0, 1, 0.01, 0, 1, 0, 0, -1, 0, 0, 0], np.float32)]


@pytest.mark.parametrize("debug", [None, 4])
@pytest.mark.parametrize("k", range(len(_GENERAL_XFS)))
def test_coarse_general_transforms(k, debug):
    xf = _GENERAL_XFS[k]
    s = H.GpuScene("rabbit_70k", 240, 136, kernel=3, debug=debug)
    argb, hit, cnt = s.render(0, xform=xf, count=True)
    oargb, ohit, ocnt = H.oracle_render("rabbit_70k", 240, 136, 0, xform=xf)
    _assert_same((argb, hit), (oargb, ohit), f"xf {k} debug {debug}")
    _counters_match(cnt, ocnt, 3)
    argb2, hit2, _ = s.render(0, xform=xf)
    _assert_same((argb2, hit2), (oargb, ohit), f"xf {k} debug {debug} (no counters)")


# A root box at the eye's depth (round 6): an object moved beside or around
# the camera (the keyboard path's `--animate` poses reach it).  Its rectangle
# comes from the box's part in front of the eye (root_rect_clipped), and an
# eye inside the box sends every group to the coarse kernel's exact root test
# (no ray enters such a box, TD/Trixel.cu:95).  Debug bit 8192: the previous
# whole-frame fine grid.  The frames are the oracle's either way.
def _xlate(t, deg=0.0):
    x = _rot_y(deg)
    x[3], x[7], x[11] = t
    return x


_STRADDLE = [((0.10, 0.0, -0.958463), 0.0), ((-0.067, 0.0, -0.953463), 0.0), ((0.0, 0.075, -0.958463), 0.0),
             ((0.0, -0.095, -0.948463), 0.0), ((0.10, 0.0, -0.958463), 12.0), ((0.03, 0.0, -0.998463), 0.0),
             ((0.0, -0.0101542, -0.998463), 30.0), ((-0.5, 0.0, -1.1), 0.0), ((-0.5, 0.0, -1.1), -20.0)]


@pytest.mark.parametrize("k", range(len(_STRADDLE)))
def test_root_box_at_eye_depth(k):
    t, deg = _STRADDLE[k]
    xf = _xlate(t, deg)
    from cpp_cuda_raytracer_dev_amd import _lib
    oargb, ohit, ocnt = H.oracle_render("rabbit_70k", 240, 136, 0, xform=xf)
    fine = {}
    for debug in (None, 8192):
        s = H.GpuScene("rabbit_70k", 240, 136, kernel=3, debug=debug)
        argb, hit, cnt = s.render(0, xform=xf, count=True)
        _assert_same((argb, hit), (oargb, ohit), f"straddle {k} debug {debug}")
        _counters_match(cnt, ocnt, 3)
        argb2, hit2, _ = s.render(0, xform=xf, shadow=True)
        sargb, shit, _ = H.oracle_render("rabbit_70k", 240, 136, 0, xform=xf, shadow=True)
        _assert_same((argb2, hit2), (sargb, shit), f"straddle {k} debug {debug} shadow")
        fine[debug] = s.cam.get_option(_lib.RT_OPT_FINE_TILES)
        s.close()
    # the whole frame was fine before; the clipped rectangle (or none, for an
    # eye inside the box) leaves fewer fine tiles
    assert fine[8192] == (240 // 8) * (136 // 8), fine
    assert fine[None] < fine[8192], fine


def test_camera_inside_root_box():
    """An untransformed object with the eye inside its root box: no ray enters
    the box, the groups run the coarse kernel's exact test, not fine units."""
    from cpp_cuda_raytracer_dev_amd import _lib
    pose = dict(pos=(-0.01, 0.11, -0.02), look_at=(-0.01, 0.11, 1.0))
    for debug in (None, 8192):
        s = H.GpuScene("rabbit_70k", 240, 136, cam_kw=pose, kernel=3, debug=debug)
        argb, hit, cnt = s.render(0, count=True)
        oargb, ohit, ocnt = H.oracle_render("rabbit_70k", 240, 136, 0, cam_kw=pose)
        _assert_same((argb, hit), (oargb, ohit), f"inside debug {debug}")
        _counters_match(cnt, ocnt, 3)
        assert (ohit < 0).all()
        tiles = s.cam.get_option(_lib.RT_OPT_FINE_TILES)
        assert tiles == (0 if debug is None else (240 // 8) * (136 // 8)), (debug, tiles)
        s.close()


@pytest.mark.parametrize("debug", [None, 4])
def test_coarse_shadow(debug):
    s = H.GpuScene("dragon", 960, 540, kernel=3, debug=debug)
    argb, hit, cnt = s.render(0, count=True, shadow=True)
    oargb, ohit, ocnt = H.oracle_render("dragon", 960, 540, 0, shadow=True)
    _assert_same((argb, hit), (oargb, ohit), f"coarse shadow debug {debug}")
    _counters_match(cnt, ocnt, 3)


@pytest.mark.parametrize("debug", [None, 4])
@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_coarse_band_tiles(nranks, debug):
    import torch
    from cpp_cuda_raytracer_dev_amd import raytracer as R
    w, h = 960, 540
    s = H.GpuScene("dragon", w, h, kernel=3, coarse=0)
    full, _, _ = s.render(0)
    t = H.GpuScene("dragon", w, h, kernel=3, debug=debug)
    npk = R.packed_pixels(w, h, nranks)
    gathered = torch.zeros(nranks * npk, dtype=torch.int32, device="cuda:0")
    for r in range(nranks):
        t.cam.render_into(gathered[r * npk:(r + 1) * npk], mode=0, tile=(nranks, r))
    frame = torch.zeros(w * h, dtype=torch.int32, device="cuda:0")
    R.unpack_bands(0, w, h, nranks, gathered, frame)
    torch.cuda.synchronize()
    assert (frame.cpu().numpy().view(np.uint32) == full).all()


# ------------------------------------------------------ cost-ordered tiles
# Tile order 3 dispatches fine tiles heaviest-first by the pool iterations an
# earlier frame measured (read back asynchronously every few frames).  Any
# permutation gives the same frame; these tests run enough frames for the
# feedback to reorder the tiles, then compare with the oracle.
@pytest.mark.parametrize("order", [3, 4])
@pytest.mark.parametrize("rays", [16, 8])
@pytest.mark.parametrize("name,w,h", [("dragon", 960, 540), ("rabbit_70k", 320, 180)])
def test_cost_order_feedback(name, w, h, rays, order):
    import torch
    s = H.GpuScene(name, w, h, kernel=3, tile_order=order, rays=rays)
    oargb, ohit, ocnt = H.oracle_render(name, w, h, 0)
    out = torch.zeros(w * h, dtype=torch.int32, device="cuda:0")
    st = torch.cuda.Stream()
    for _ in range(60):
        s.cam.render_into(out, mode=0, stream=st.cuda_stream)
        st.synchronize()  # lets the cost sample arrive between frames
    assert (out.cpu().numpy().view(np.uint32) == oargb).all()
    argb, hit, cnt = s.render(0, count=True)
    _assert_same((argb, hit), (oargb, ohit), f"{name} cost order")
    _counters_match(cnt, ocnt, 3)
    # the order in use is a permutation of the fine tiles
    for _ in range(3):
        s.cam.render_into(out, mode=0, stream=st.cuda_stream)
    st.synchronize()
    assert (out.cpu().numpy().view(np.uint32) == oargb).all()


@pytest.mark.parametrize("order", [3, 4])
def test_cost_order_pose_change(order):
    """A new camera transform changes the fine grid; the stale cost sample is dropped."""
    import torch
    s = H.GpuScene("rabbit_70k", 320, 180, kernel=3, tile_order=order)
    out = torch.zeros(320 * 180, dtype=torch.int32, device="cuda:0")
    for i in range(40):
        xf = _rot_y(float(i % 5) * 7.0, (0.01 * (i % 3), 0.0, 0.0))
        s.obj.quat.rot_m = np.asarray(xf, np.float32).reshape(3, 4)
        s.cam.render_into(out, xform=s.obj.quat.xform(), mode=0)
    xf = _rot_y(14.0, (0.01, 0.0, 0.0))
    argb, hit, _ = s.render(0, xform=xf)
    oargb, ohit, _ = H.oracle_render("rabbit_70k", 320, 180, 0, xform=xf)
    _assert_same((argb, hit), (oargb, ohit), "cost order after pose changes")


# ------------------------------------------------------- frame delivery
# frames copied to pinned host memory on a copy stream
# while the next frame renders (rt_pinned_alloc / rt_frame_copy_async).
def test_frame_delivery_pinned_double_buffered():
    import torch
    from cpp_cuda_raytracer_dev_amd import raytracer as R
    w, h = 320, 180
    s = H.GpuScene("rabbit_70k", w, h, kernel=3)
    xfs = [_rot_y(float(a), (0.0, 0.0, 0.005 * k)) for k, a in enumerate((0, 7, 14, 21, 28))]
    want = [H.oracle_render("rabbit_70k", w, h, 0, xform=xf)[0] for xf in xfs]
    dev = torch.device("cuda:0")
    outs = [torch.zeros(w * h, dtype=torch.int32, device=dev) for _ in range(2)]
    pf = R.PinnedFrames(w * h, 2)
    rs, cs = torch.cuda.Stream(), torch.cuda.Stream()
    rendered = [torch.cuda.Event() for _ in range(2)]
    copied = [torch.cuda.Event() for _ in range(2)]
    for k in range(2):
        copied[k].record(cs)
    got = []
    for i, xf in enumerate(xfs):
        k = i % 2
        if i >= 2:
            copied[k].synchronize()
            got.append(pf.frames[k].copy())  # frame i - 2, before its buffer is reused
        rs.wait_event(copied[k])
        s.cam.render_into(outs[k], xform=xf, mode=0, stream=rs.cuda_stream)
        rendered[k].record(rs)
        cs.wait_event(rendered[k])
        pf.copy_async(k, 0, outs[k], stream=cs.cuda_stream)
        copied[k].record(cs)
    torch.cuda.synchronize()
    for i in range(len(xfs) - 2, len(xfs)):
        got.append(pf.frames[i % 2].copy())
    pf.close()
    assert len(got) == len(xfs)
    for i, (g, wnt) in enumerate(zip(got, want)):
        assert (g == wnt).all(), f"delivered frame {i} differs from the oracle"


# ------------------------------------------------------- binary PLY mesh
# 3_walls.ply (the reference's binary file, read by rt_read_ply's binary
# path; fixture bytes in tests/golden/meshes/3_walls.npz) through the KD
# kernels, two poses that see its walls.
@pytest.mark.parametrize("kernel", [2, 3])
@pytest.mark.parametrize("pose", [dict(pos=(-100.0, 20.0, -50.0), look_at=(-307.0, 0.0, 2.0)),
                                  dict(pos=(-150.0, -60.0, 120.0), look_at=(-307.0, 10.0, 0.0))])
def test_binary_mesh_3_walls(pose, kernel):
    s = H.GpuScene("3_walls", 160, 90, cam_kw=pose, kernel=kernel)
    argb, hit, cnt = s.render(0, count=True)
    oargb, ohit, ocnt = H.oracle_render("3_walls", 160, 90, 0, cam_kw=pose)
    assert (ohit >= 0).sum() > 1000
    _assert_same((argb, hit), (oargb, ohit), "3_walls")
    _counters_match(cnt, ocnt, kernel)


# ------------------------------------------------------------ object motion
# the keyboard transform path (rt_object_*) drives the
# rot_m of consecutive frames; each frame equals the oracle's render with the
# oracle's own restatement of the motion (oracle/motion.py).
@pytest.mark.parametrize("kernel", [2, 3])
def test_animated_key_sequence(kernel):
    from cpp_cuda_raytracer_dev_amd import raytracer as R
    from oracle import motion as M
    from oracle import np_oracle as N
    s = H.GpuScene("rabbit_70k", 320, 180, kernel=kernel)
    cam = N.camera(320, 180)
    ref = M.Motion(cam["pos"], cam["n"], cam["u"])
    seq = [R.KEY_W, R.KEY_R, R.KEY_W | R.KEY_Q, R.KEY_R, R.KEY_T | R.KEY_S, R.KEY_E, R.KEY_R | R.KEY_W, R.KEY_Q,
           R.KEY_T, R.KEY_T, R.KEY_W, R.KEY_R]
    hits = []
    for i, keys in enumerate(seq):
        s.obj.key_tick(keys)
        ref.tick(keys)
        xf = ref.xform()
        assert (s.obj.quat.xform().view(np.uint32) == xf.view(np.uint32)).all()
        if i % 3 == 2:
            argb, hit, _ = s.render(0)
            oargb, ohit, _ = H.oracle_render("rabbit_70k", 320, 180, 0, xform=xf)
            _assert_same((argb, hit), (oargb, ohit), f"tick {i} keys {keys}")
            hits.append(int((ohit >= 0).sum()))
    assert max(hits) > 100


@pytest.mark.parametrize("kernel", [2, 3])
def test_animated_key_sequence_display(kernel):
    """rt_render_display over a moving key sequence: the displayed frames
    (the reference's window, ghosting included: TD/WinMain.cpp:212-237,
    TD/Camera.cu:27-61,77-84,98) equal oracle.c's orc_window_frame
    composition bit for bit, and the clean buffer is the oracle's frame."""
    import torch
    from oracle import _oracle as O
    from tests.test_motion import GHOST_KEYS, ghost_sequence
    w, h = 160, 90
    frames, hits, poses = ghost_sequence(w=w, h=h)
    s = H.GpuScene("rabbit_70k", w, h, kernel=kernel)
    dev = torch.device("cuda:0")
    clean = torch.zeros(w * h, dtype=torch.int32, device=dev)  # init_cam_mem_cuda's zeroed buffer
    shown = torch.full((w * h,), -1, dtype=torch.int32, device=dev)
    win = O.Window(w * h)
    ghosts = 0
    for k, keys in enumerate(GHOST_KEYS):
        s.obj.key_tick(keys)
        xf = s.obj.quat.xform()
        assert (xf.view(np.uint32) == np.asarray(poses[k], np.float32).view(np.uint32)).all()
        s.cam.render_display(clean, shown, xform=xf)
        torch.cuda.synchronize()
        want = win.frame(frames[k], hits[k])
        got = shown.cpu().numpy().view(np.uint32)
        assert (got == want).all(), (k, int((got != want).sum()))
        assert (clean.cpu().numpy().view(np.uint32) == frames[k]).all(), k
        if k:
            ghosts += int(((hits[k - 1] >= 0) & (hits[k] < 0)).sum())
    assert ghosts > 20


@pytest.mark.parametrize("scene,w,h", [("dragon", 480, 270), ("rabbit_70k", 320, 180)])
def test_held_fine_region_same_frames(scene, w, h):
    """A drifting object: renders keep the fine region they chose while the
    exact one stays inside it (set_fine_region's hold); every frame equals a
    camera rendering the exact region (debug bit 256) and, at a few poses,
    the oracle."""
    a = H.GpuScene(scene, w, h)
    b = H.GpuScene(scene, w, h, debug=256)
    rng = np.random.default_rng(5)
    off = np.zeros(3, np.float32)
    for k in range(24):
        off += rng.normal(0, 0.002, 3).astype(np.float32)
        ang = 0.01 * k
        c, s_ = np.float32(np.cos(ang)), np.float32(np.sin(ang))
        xf = np.array([c, 0, s_, off[0], 0, 1, 0, off[1], -s_, 0, c, off[2]], np.float32)
        ga, ha, _ = a.render(0, xform=xf)
        gb, hb, _ = b.render(0, xform=xf)
        _assert_same((ga, ha), (gb, hb), f"pose {k}")
        if k % 8 == 7:
            oargb, ohit, _ = H.oracle_render(scene, w, h, 0, xform=xf)
            _assert_same((ga, ha), (oargb, ohit), f"pose {k} vs oracle")


def test_animated_shadow_frame():
    from cpp_cuda_raytracer_dev_amd import raytracer as R
    from oracle import motion as M
    from oracle import np_oracle as N
    s = H.GpuScene("rabbit_70k", 320, 180, kernel=3)
    cam = N.camera(320, 180)
    ref = M.Motion(cam["pos"], cam["n"], cam["u"])
    for keys in (R.KEY_R, R.KEY_W, R.KEY_Q):
        s.obj.key_tick(keys)
        ref.tick(keys)
    argb, hit, _ = s.render(0, shadow=True)
    oargb, ohit, _ = H.oracle_render("rabbit_70k", 320, 180, 0, xform=ref.xform(), shadow=True)
    assert (ohit >= 0).sum() > 100
    _assert_same((argb, hit), (oargb, ohit), "animated shadow frame")


def test_headless_driver_key_sequence(tmp_path):
    """tools/rt_headless (the WinMain replacement over include/rt_facade.hpp)
    with a held-key sequence: its last frame equals the oracle's render after
    the same ticks."""
    import os
    import subprocess
    from cpp_cuda_raytracer_dev_amd import scenes
    from oracle import motion as M
    from oracle import np_oracle as N
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "rt_headless")
    if not os.path.exists(exe):
        pytest.skip("tools/rt_headless not built (python -m cpp_cuda_raytracer_dev_amd.build)")
    v, a, ix = scenes.fixture_mesh("rabbit_70k")
    ply = tmp_path / "rabbit.ply"
    scenes.write_ply(str(ply), v, np.asarray(ix, np.int32).reshape(-1, 3))
    ppm = tmp_path / "out.ppm"
    w, h, frames, keys = 320, 180, 5, "R+W.QT"
    r = subprocess.run([exe, str(ply), "0", str(w), str(h), str(frames), str(ppm), "0", keys], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    img = np.frombuffer(ppm.read_bytes()[len(f"P6\n{w} {h}\n255\n"):], np.uint8).reshape(h, w, 3)[::-1]
    got = (img[..., 0].astype(np.uint32) << 16) | (img[..., 1].astype(np.uint32) << 8) | img[..., 2]
    cam = N.camera(w, h)
    ref = M.Motion(cam["pos"], cam["n"], cam["u"])
    ticks = [M.KEY_R | M.KEY_W, 0, M.KEY_Q, M.KEY_T]
    for f in range(frames):
        ref.tick(ticks[f % len(ticks)])
    oargb, ohit, _ = H.oracle_render("rabbit_70k", w, h, 0, xform=ref.xform())
    assert (ohit >= 0).sum() > 100
    assert (got.reshape(-1) == oargb).all()


@pytest.mark.parametrize("order", [0, 1, 2, 3])
def test_shadow_push_orders(order):
    """Every any-hit push order renders the identical shadow frame (no counting:
    the walks stop at their first occluder, so the order changes the work)."""
    from cpp_cuda_raytracer_dev_amd import _lib
    s = H.GpuScene("dragon", 960, 540, kernel=3)
    s.cam.set_option(_lib.RT_OPT_SHADOW_ORDER, order)
    argb, hit, _ = s.render(0, shadow=True)
    oargb, ohit, _ = H.oracle_render("dragon", 960, 540, 0, shadow=True)
    _assert_same((argb, hit), (oargb, ohit), f"shadow push order {order}")
    assert s.cam.get_option(_lib.RT_OPT_SHADOW_ORDER) == order


def test_shadow_push_order_timed():
    """The timed choice (default): a round of trial frames, then the fastest
    order; every frame along the way is exact."""
    import torch
    from cpp_cuda_raytracer_dev_amd import _lib, raytracer as R
    w, h = 480, 270
    s = H.GpuScene("dragon", w, h, kernel=3)
    oargb, _, _ = H.oracle_render("dragon", w, h, 0, shadow=True)
    out = torch.zeros(w * h, dtype=torch.int32, device="cuda:0")
    for i in range(20):
        s.cam.render_into(out, mode=0, flags=R.RT_FLAG_SHADOW)
        torch.cuda.synchronize()
        assert (out.cpu().numpy().view(np.uint32) == oargb).all(), f"frame {i}"
    assert s.cam.get_option(_lib.RT_OPT_SHADOW_ORDER) in (0, 1, 2, 3)
    with pytest.raises(_lib.RtError):
        s.cam.set_option(_lib.RT_OPT_SHADOW_ORDER, 4)


@pytest.mark.parametrize("order", [0, 3])
def test_shadow_counted_stop_at_occluder(order):
    """Debug bit 16 counts the walk a timed shadow frame does (stops at the
    first occluder): fewer visits than the full walk, the same frame."""
    from cpp_cuda_raytracer_dev_amd import _lib
    s = H.GpuScene("dragon", 480, 270, kernel=3)
    s.cam.set_option(_lib.RT_OPT_SHADOW_ORDER, order)
    argb, hit, full = s.render(0, count=True, shadow=True)
    s.cam.set_option(_lib.RT_OPT_DEBUG, 16)
    argb2, hit2, cut = s.render(0, count=True, shadow=True)
    assert (argb == argb2).all() and (hit == hit2).all()
    assert cut[0] < full[0] and cut[1] <= full[1] and cut[3] == full[3]


@pytest.mark.parametrize("w,h,nranks", [(81, 45, 3), (33, 9, 2), (64, 20, 8), (7, 130, 5)])
def test_unpack_bands_shapes(w, h, nranks):
    """k_unpack's row copy (16-byte pieces when w % 4 == 0, else words) against
    the numpy inverse of the packing, on random words."""
    import torch
    from cpp_cuda_raytracer_dev_amd import raytracer as R, distributed as D
    npk = R.packed_pixels(w, h, nranks)
    rng = np.random.default_rng(w * 1000 + h)
    g = rng.integers(0, 2**32, nranks * npk, dtype=np.uint64).astype(np.uint32)
    dev = torch.device("cuda:0")
    gathered = torch.from_numpy(g.view(np.int32)).to(dev)
    frame = torch.full((w * h,), -1, dtype=torch.int32, device=dev)
    R.unpack_bands(0, w, h, nranks, gathered, frame)
    torch.cuda.synchronize()
    assert (frame.cpu().numpy().view(np.uint32) == D.unpack_bands_numpy(g, w, h, nranks)).all()
    # a misaligned frame pointer takes the word path
    frame2 = torch.full((w * h + 1,), -1, dtype=torch.int32, device=dev)
    R.unpack_bands(0, w, h, nranks, gathered, frame2[1:])
    torch.cuda.synchronize()
    assert (frame2[1:].cpu().numpy().view(np.uint32) == D.unpack_bands_numpy(g, w, h, nranks)).all()


@pytest.mark.parametrize("direct", [False, True])
@pytest.mark.parametrize("scene,w,h,nranks,moved", [("dragon", 1920, 1080, 2, False), ("dragon", 1920, 1080, 8, False),
                                                     ("rabbit_70k", 81, 45, 3, False), ("dragon", 960, 540, 4, True),
                                                     ("dragon", 960, 540, 1, False)])
def test_rect_gather_single_gpu(scene, w, h, nranks, moved, direct):
    """The rectangle gather of rt_comm_gather_frame, every rank simulated on
    one GPU: each rank's tile render -> rt_pack_rect -> (the peers' parts back
    to back) -> rt_unpack_rect with rank 0's own buffer equals the full frame.
    A moved object has no background proof: the rectangle is the whole frame.
    direct: rank 0 renders its bands into the (poisoned) frame itself
    (RT_FLAG_FRAME_OUT, what rt_run_frames does) and the assembly leaves them."""
    import ctypes as C
    import torch
    from cpp_cuda_raytracer_dev_amd import _lib, raytracer as R
    s = H.GpuScene(scene, w, h)
    xf = None
    if moved:
        xf = np.array([1, 0, 0, 0.01, 0, 1, 0, 0, 0, 0, 1, 0.02], np.float32)
        s.obj.quat.rot_m = xf.reshape(3, 4)
    full, _, _ = s.render(0, xform=xf)
    rect = np.zeros(4, np.int32)
    _lib.call("rt_frame_rect", s.cam._h, _lib.ptr(xf), 0, nranks, _lib.ptr(rect))
    nbands = (h + 7) // 8
    if moved:
        assert tuple(rect) == (0, w, 0, nbands)
    elif w >= 960:  # small frames: the widened projection may cover everything
        assert 0 < (rect[1] - rect[0]) * (rect[3] - rect[2]) < w * nbands
    npk = R.packed_pixels(w, h, nranks)
    dev = torch.device("cuda:0")
    locs = [torch.zeros(npk, dtype=torch.int32, device=dev) for _ in range(nranks)]
    for r in range(nranks):
        s.cam.render_into(locs[r], xform=xf, mode=0, tile=(nranks, r))
    counts = [int(_lib.lib().rt_rect_pixels(w, h, nranks, r, _lib.ptr(rect))) for r in range(nranks)]
    assert min(counts) >= 0
    peers = torch.zeros(max(1, sum(counts[1:])), dtype=torch.int32, device=dev)
    off = 0
    for r in range(1, nranks):
        if counts[r]:
            _lib.call("rt_pack_rect", 0, w, h, nranks, r, _lib.ptr(rect), _lib.ptr(locs[r]),
                      C.c_void_p(peers.data_ptr() + 4 * off), None)
        off += counts[r]
    frame = torch.full((w * h,), -1, dtype=torch.int32, device=dev)
    if direct:
        s.cam.render_into(frame, xform=xf, mode=0, flags=R.RT_FLAG_FRAME_OUT, tile=(nranks, 0))
    _lib.call("rt_unpack_rect", 0, w, h, nranks, _lib.ptr(rect), _lib.ptr(frame if direct else locs[0]),
              _lib.ptr(peers), _lib.ptr(frame), None)
    torch.cuda.synchronize()
    got = frame.cpu().numpy().view(np.uint32)
    assert (got == full).all(), int((got != full).sum())


@pytest.mark.parametrize("scene,w,h,moved,rays,coarse", [("dragon", 1920, 1080, False, 0, 8),
                                                         ("knot", 1920, 1080, False, 0, 8),
                                                         ("rabbit_70k", 960, 540, False, 8, 4),
                                                         ("dragon", 960, 540, True, 0, 8),
                                                         ("rabbit_70k", 81, 45, False, 0, 8)])
def test_frame_rect_host_equals_camera(scene, w, h, moved, rays, coarse):
    """rt_frame_rect_host from the host-side inputs (the basis of
    rt_camera_basis, the root box minus the camera position, the options: what
    tests/test_distributed_gloo.py's ranks derive without a GPU) equals the
    device camera's rt_frame_rect for every rank count; rt_camera_frame_geometry
    reports the same inputs; the host pack / assembly equal the device ones."""
    import ctypes as C
    import torch
    from cpp_cuda_raytracer_dev_amd import _lib, raytracer as R
    from cpp_cuda_raytracer_dev_amd.distributed import frame_geometry, frame_rect_host
    s = H.GpuScene(scene, w, h, rays=rays, coarse=coarse)
    xf = np.array([1, 0, 0, 0.01, 0, 1, 0, 0, 0, 0, 1, 0.02], np.float32) if moved else None
    g = _lib.RtFrameGeometry()
    _lib.call("rt_camera_frame_geometry", s.cam._h, C.byref(g))
    pos, la, up = (0.0, 0.1, -1.0), (0.0, 0.1, 0.0), (0.0, 1.0, 0.0)
    basis = R.camera_basis(w, h, R.film_w(w, h), np.float32(.024), np.float32(.055), pos, la, up)
    root = H.product_tree(scene)[0]
    p = np.float32(pos)
    box = [np.float32(root[k]) - p[i // 2] for i, k in enumerate(("x0", "x1", "y0", "y1", "z0", "z1"))]
    hg = frame_geometry(w, h, basis, box, bool(root["is_leaf"]), kernel=3, rays=rays, coarse=coarse)
    assert bytes(hg) == bytes(g)
    for nranks in (1, 2, 3, 4, 8):
        rect = np.zeros(4, np.int32)
        _lib.call("rt_frame_rect", s.cam._h, _lib.ptr(xf), 0, nranks, _lib.ptr(rect))
        assert frame_rect_host(hg, xf, 0, nranks) == tuple(int(v) for v in rect), nranks
    # host and device pack / assembly of the same packed buffers
    nranks = 4
    rect = np.array(frame_rect_host(hg, xf, 0, nranks), np.int32)
    npk = R.packed_pixels(w, h, nranks)
    dev = torch.device("cuda:0")
    locs = [torch.zeros(npk, dtype=torch.int32, device=dev) for _ in range(nranks)]
    for r in range(nranks):
        s.cam.render_into(locs[r], xform=xf, mode=0, tile=(nranks, r))
    torch.cuda.synchronize()
    counts = [int(_lib.lib().rt_rect_pixels(w, h, nranks, r, _lib.ptr(rect))) for r in range(nranks)]
    hpeers = np.zeros(max(1, sum(counts[1:])), np.uint32)
    off = 0
    for r in range(1, nranks):
        part = np.zeros(max(1, counts[r]), np.uint32)
        loc = locs[r].cpu().numpy().view(np.uint32).copy()
        _lib.call("rt_pack_rect_host", w, h, nranks, r, _lib.ptr(rect), _lib.ptr(loc), _lib.ptr(part))
        dpart = torch.zeros(max(1, counts[r]), dtype=torch.int32, device=dev)
        if counts[r]:
            _lib.call("rt_pack_rect", 0, w, h, nranks, r, _lib.ptr(rect), _lib.ptr(locs[r]), _lib.ptr(dpart), None)
        torch.cuda.synchronize()
        assert (dpart.cpu().numpy().view(np.uint32)[:counts[r]] == part[:counts[r]]).all()
        hpeers[off:off + counts[r]] = part[:counts[r]]
        off += counts[r]
    frame = np.zeros(w * h, np.uint32)
    loc0 = locs[0].cpu().numpy().view(np.uint32).copy()
    _lib.call("rt_unpack_rect_host", w, h, nranks, _lib.ptr(rect), _lib.ptr(loc0), _lib.ptr(hpeers), _lib.ptr(frame))
    full, _, _ = s.render(0, xform=xf)
    assert (frame == full).all(), int((frame != full).sum())


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("nranks", [1, 2, 3, 8])
def test_frame_out_tile_rows(nranks, mode):
    """RT_FLAG_FRAME_OUT: a rank's bands land on their frame rows of a w*h
    buffer (colour and hit), every other row untouched; all ranks together
    give the full frame."""
    import torch
    s = H.GpuScene("rabbit_70k", 81, 45)
    full, fhit, _ = s.render(mode)
    dev = torch.device("cuda:0")
    w, h = 81, 45
    frame = torch.full((w * h,), -1, dtype=torch.int32, device=dev)
    hit = torch.full((w * h,), -7, dtype=torch.int64, device=dev)
    rows = np.arange(h) // 8 % nranks
    for r in range(nranks):
        s.cam.render_into(frame, hit, mode=mode, flags=R.RT_FLAG_FRAME_OUT | R.RT_FLAG_WRITE_HIT, tile=(nranks, r))
        torch.cuda.synchronize()
        got = frame.cpu().numpy().view(np.uint32).reshape(h, w)
        gh = hit.cpu().numpy().reshape(h, w)
        done = rows <= r
        assert (got[done] == full.reshape(h, w)[done]).all()
        assert (gh[done] == fhit.reshape(h, w)[done]).all()
        assert (got[~done] == 0xFFFFFFFF).all() and (gh[~done] == -7).all()


def test_native_comm_world1():
    """rt_comm_* end to end in a one-rank group: RCCL resolved at run time, the
    id broadcast, the communicator, rt_comm_gather_frame's in-place slot 0 +
    unpack on a side stream, pipelined over two buffer sets.  Each frame has
    its own object transform and poisoned render target, and a set is reused
    only once its gather has read it ('sent' events), so a frame gathered
    from the wrong set or before its render shows."""
    import os
    import tempfile
    import torch
    import torch.distributed as dist
    from cpp_cuda_raytracer_dev_amd import _lib
    from cpp_cuda_raytracer_dev_amd.distributed import NativeFrameGather
    assert _lib.lib().rt_comm_available() == 1
    w, h = 320, 180
    s = H.GpuScene("rabbit_70k", w, h)
    poses = [_rot_y(0.0), _rot_y(7.0), _rot_y(-5.0, (0.004, 0.0, 0.0)), _rot_y(11.0), _rot_y(0.0, (0.0, 0.003, 0.0))]
    fulls = [s.render(0, xform=xf)[0] for xf in poses]
    fd, path = tempfile.mkstemp()
    os.close(fd)
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=0, world_size=1)
    try:
        dev = torch.device("cuda:0")
        ng = NativeFrameGather(dist, w, h, dev, nbuf=2)
        rs, cs = torch.cuda.Stream(), torch.cuda.Stream()
        rendered = [torch.cuda.Event() for _ in range(2)]
        sent = [torch.cuda.Event() for _ in range(2)]
        got = []
        for j, xf in enumerate(poses):
            k = j % 2
            rs.wait_event(sent[k])  # the gather that last read set k is done
            with torch.cuda.stream(rs):
                ng.local[k].fill_(0x7BADBEEF)
            s.cam.render_into(ng.local[k], xform=xf, mode=0, stream=rs.cuda_stream)
            rendered[k].record(rs)
            cs.wait_event(rendered[k])
            ng.gather(k, s.cam, xf, 0, cs.cuda_stream)
            sent[k].record(cs)
            if j >= 1:  # frame j-1's set: check it once its gather is done
                sent[(j - 1) % 2].synchronize()
                got.append(ng.frames[(j - 1) % 2].cpu().numpy().view(np.uint32).copy())
        torch.cuda.synchronize()
        got.append(ng.frames[(len(poses) - 1) % 2].cpu().numpy().view(np.uint32).copy())
        for j, (g, f) in enumerate(zip(got, fulls)):
            assert (g == f).all(), f"frame {j}"
        x0, x1, b0, b1 = ng.verify(s.cam, None, 0)
        assert (x1 - x0) * (b1 - b0) * 8 < w * h  # the fused render proves part of the frame background
        # the native frame loop over the same communicator: identical frames
        loop = R.FrameLoop(s.cam, ng.local, mode=0, render_stream=rs.cuda_stream, comm=ng,
                           comm_stream=cs.cuda_stream, event_every=2)
        ms, n, host = loop.run(9)
        assert n == 5 and ms > 0 and host > 0
        assert (ng.frames[loop.last_set()].cpu().numpy().view(np.uint32) == fulls[0]).all()
        # two frames in flight on the library's lanes, gathers on its comm
        # lane: every set's gathered frame is whole
        for f in ng.frames:
            f.fill_(0x7BADBEEF)
        torch.cuda.synchronize()
        loop = R.FrameLoop(s.cam, ng.local, mode=0, render_stream=rs.cuda_stream, comm=ng,
                           comm_stream=cs.cuda_stream, event_every=3, inflight=2)
        ms, n, host = loop.run(12)
        assert n == 4 and ms > 0
        for f in ng.frames:
            assert (f.cpu().numpy().view(np.uint32) == fulls[0]).all()
        # with a tile, rank 0 renders straight into each set's frame
        # (RT_FLAG_FRAME_OUT) and its lanes share no events: one pose per
        # frame, poisoned frames, 1 and 2 frames in flight
        xfs = np.stack([np.asarray(xf, np.float32).reshape(12) for xf in poses])
        for inflight in (1, 2):
            for f in ng.frames:
                f.fill_(0x7BADBEEF)
            torch.cuda.synchronize()
            loop = R.FrameLoop(s.cam, ng.local, mode=0, tile=(1, 0), render_stream=rs.cuda_stream, comm=ng,
                               comm_stream=cs.cuda_stream, inflight=inflight, xforms=xfs)
            loop.run(len(poses) + 2)  # frames 0..6 at poses j % 5: the sets end with frames 5 and 6
            for j in (len(poses), len(poses) + 1):
                got = ng.frames[j % 2].cpu().numpy().view(np.uint32)
                assert (got == fulls[j % len(poses)]).all(), (inflight, j)
        ng.close()
    finally:
        dist.destroy_process_group()
        if os.path.exists(path):  # the file store removes it itself
            os.unlink(path)


@pytest.mark.gpu
def test_shim_ranks_gather():
    """the library's own N > 1 gather (csrc/comm.cpp:
    rank 0's ncclRecv loop and direct-path assembly, the peers' pack +
    ncclSend) and rt_run_frames' render / comm event ordering with peers
    present, run by N = 2, 4, 8 ranks as threads of one process on one GPU
    through the test-only RCCL shim (tests/rccl_shim, loaded via RT_RCCL_LIB):
    dragon stand-in 1920x1080, two frames in flight, four buffer sets, one
    object pose per frame.  Every buffer set rank 0 assembled equals the
    oracle's frame at its pose (the committed hash for the identity pose, a
    live oracle render for the moved ones) and every rank's device error
    word is 0.  This is not an N > 1 hardware measurement."""
    import json
    import os
    import subprocess
    import sys
    from tests.rccl_shim import build as shim
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RT_RCCL_LIB=shim.build())
    r = subprocess.run([sys.executable, "-u", os.path.join(root, "tests", "shim_ranks.py"), "--nranks", "2,4,8",
                        "--frames", "24"], cwd=root, env=env, capture_output=True, text=True, timeout=110)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, f"no result (exit {r.returncode}): {r.stdout[-2000:]} {r.stderr[-2000:]}"
    out = json.loads(lines[-1])
    print(json.dumps(out))
    assert r.returncode == 0 and out["ok"], out
    assert [g["nranks"] for g in out["groups"]] == [2, 4, 8]
    for g in out["groups"]:
        assert g["device_err"] == [0] * g["nranks"], g
        assert all(s["equal"] for s in g["sets"]), g
        assert {s["pose"] for s in g["sets"]} - {0}, "a moved pose is checked"


@pytest.mark.gpu
def test_shim_ranks_gather_c5():
    """BASELINE config C5 (happy stand-in 3840x2160, one
    shadow ray per hit, 8 ranks) through the library's own N > 1 gather
    (csrc/comm.cpp) via the test-only RCCL shim: 4K rectangle parts of up to
    4.1 MB per rank and shadowed frames go through rank 0's ncclRecv loop and
    assembly.  Identity pose; every buffer set rank 0 assembled hashes to the
    committed oracle frame happy_3840x2160_m0_shadow, every rank's device
    error word is 0.  Not an N > 1 hardware measurement."""
    import json
    import os
    import subprocess
    import sys
    from tests.rccl_shim import build as shim
    ent = H.frame_hashes()["happy_3840x2160_m0_shadow"]
    if not H.mesh_matches(ent):
        pytest.skip("the happy stand-in's mesh differs on this host (numpy transcendentals)")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RT_RCCL_LIB=shim.build())
    r = subprocess.run([sys.executable, "-u", os.path.join(root, "tests", "shim_ranks.py"), "--nranks", "8",
                        "--scene", "happy", "--width", "3840", "--height", "2160", "--shadow", "--identity-only",
                        "--frames", "16"], cwd=root, env=env, capture_output=True, text=True, timeout=110)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, f"no result (exit {r.returncode}): {r.stdout[-2000:]} {r.stderr[-2000:]}"
    out = json.loads(lines[-1])
    print(json.dumps(out))
    assert r.returncode == 0 and out["ok"], out
    (g,) = out["groups"]
    assert g["nranks"] == 8 and g["device_err"] == [0] * 8, g
    assert all(s["equal"] and s["method"].startswith("sha256") for s in g["sets"]), g


def test_far_along_key_sequence_background():
    """bench.py --animate R+W.Q.T.W carries the object past
    the camera after ~500 ticks (the oracle shows background only).  The host
    then proves the box behind the eye for every pixel (rt_api.cpp
    box_behind): no fine tiles, every group filled as background by the fine
    kernel's blocks (far_all), and the N > 1 gather rectangle is empty.  The
    frames equal the oracle's at those poses (and at poses where the object is
    still in view, where the proof must not fire), for 1 and 4 ranks."""
    import bench
    import torch
    from cpp_cuda_raytracer_dev_amd import _lib
    from oracle import motion as M
    from oracle import np_oracle as N
    w, h = 640, 360
    masks = bench.key_masks("R+W.Q.T.W")
    cam = N.camera(w, h)
    ref = M.Motion(cam["pos"], cam["n"], cam["u"])
    s = H.GpuScene("dragon", w, h)
    dev = torch.device("cuda:0")
    out = torch.zeros(w * h, dtype=torch.int32, device=dev)
    hit = torch.zeros(w * h, dtype=torch.int64, device=dev)
    checked = {"visible": 0, "behind": 0}
    for i in range(2001):
        ref.tick(masks[i % len(masks)])
        if i not in (10, 40, 120, 600, 1200, 2000):
            continue
        xf = np.asarray(ref.xform(), np.float32).reshape(12)
        oargb, ohit, _ = H.oracle_render("dragon", w, h, 0, xform=xf.reshape(3, 4))
        out.fill_(0x7BADBEEF)
        s.cam.render_into(out, hit, xform=xf, flags=R.RT_FLAG_WRITE_HIT)
        torch.cuda.synchronize()
        _assert_same((out.cpu().numpy().view(np.uint32), hit.cpu().numpy()), (oargb, ohit), f"tick {i}")
        rect = np.zeros(4, np.int32)
        _lib.call("rt_frame_rect", s.cam._h, _lib.ptr(xf), 0, 4, _lib.ptr(rect))
        if (ohit >= 0).any():
            checked["visible"] += 1
            assert rect[1] > rect[0]
        elif tuple(rect) == (0, 0, 0, 0):
            checked["behind"] += 1
        # the ranks' bands of the same pose
        for r in range(4):
            loc = torch.full((R.packed_pixels(w, h, 4),), 0x5EEDF00D, dtype=torch.int32, device=dev)
            s.cam.render_into(loc, xform=xf, tile=(4, r))
            torch.cuda.synchronize()
            from cpp_cuda_raytracer_dev_amd.distributed import pack_bands_numpy
            want = pack_bands_numpy(oargb, w, h, 4, r)
            got = loc.cpu().numpy().view(np.uint32)
            # rows of the slots that hold a band of the frame (slot j: band r + 4j)
            rows = np.array([r + 4 * (y // 8) < (h + 7) // 8 and (r + 4 * (y // 8)) * 8 + y % 8 < h
                             for y in range(len(got) // w)])
            sel = np.repeat(rows, w)
            assert (got[sel] == want[sel]).all(), f"tick {i} rank {r}"
    assert checked["visible"] >= 2 and checked["behind"] >= 1, checked
    assert s.cam.device_error(reset=True) == 0


@pytest.mark.gpu
def test_multiframe_launch_grid_limit():
    """a multi-frame launch holds at most 2^32 - 1 work-items.
    The dragon fill view at 3840x2160 with 8-ray units is ~259k blocks of 256
    threads per frame, so 128 frames per launch would exceed it; the library
    takes fewer frames per launch.  Every buffer set equals a single-frame
    render of the same frame (itself checked against the oracle elsewhere)."""
    import torch
    from cpp_cuda_raytracer_dev_amd import _lib, scenes
    w, h = 3840, 2160
    s = H.GpuScene("dragon", w, h, cam_kw=scenes.view("dragon", "fill"), rays=8)
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(device=dev)
    ref = torch.zeros(w * h, dtype=torch.int32, device=dev)
    s.cam.render_into(ref, stream=st.cuda_stream)
    bufs = [torch.full((w * h,), 0x7BADBEEF, dtype=torch.int32, device=dev) for _ in range(2)]
    loop = R.FrameLoop(s.cam, bufs, mode=0, render_stream=st.cuda_stream, event_every=1,
                       inflight=_lib.RT_LOOP_MULTIFRAME)
    ms, cnt, _ = loop.run(300)
    torch.cuda.synchronize()
    assert s.cam.get_option(_lib.RT_OPT_RAYS_USED) == 8
    assert cnt == 300 and ms > 0
    for b in bufs:
        assert torch.equal(b, ref)
    assert s.cam.device_error(reset=True) == 0
    s.close()


@pytest.mark.parametrize("key", ["dragon_960x540_m0", "knot_1920x1080_m0", "dragon_1920x1080_m0"])
def test_multiframe_launch_loop(key):
    """rt_run_frames with RT_LOOP_MULTIFRAME: launches of up to 128 frames,
    each one k_trace_kd3 grid holding every frame's blocks, frame-major.
    Every buffer set holds the oracle's frame (committed hash) after 1, 3, 20
    and 200 frames, with 2 and 3 sets; the first frames before a cost order
    exists launch one at a time, and at 1920x1080 (16-ray units) a chunk of
    4 or more frames runs as two concurrent launches of half the frames each
    (RT_MF_SPLIT).  A moving object or a gather is rejected."""
    import hashlib
    import torch
    from cpp_cuda_raytracer_dev_amd import _lib
    ent = H.frame_hashes()[key]
    if not H.mesh_matches(ent):
        pytest.skip("stand-in mesh bits differ on this host")
    w, h = ent["w"], ent["h"]
    s = H.GpuScene(ent["scene"], w, h)
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(device=dev)
    for nbuf in (2, 3):
        bufs = [torch.full((w * h,), 0x7BADBEEF, dtype=torch.int32, device=dev) for _ in range(nbuf)]
        loop = R.FrameLoop(s.cam, bufs, mode=0, render_stream=st.cuda_stream, event_every=1,
                           inflight=_lib.RT_LOOP_MULTIFRAME)
        for n in (1, 3, 20, 200):
            for b in bufs:
                b.fill_(0x7BADBEEF)
            torch.cuda.synchronize()
            ms, cnt, host = loop.run(n)
            torch.cuda.synchronize()
            assert cnt == n and ms > 0
            # every set the loop wrote holds the frame (the loop's sets rotate from its sequence number)
            shas = {hashlib.sha256(b.cpu().numpy().view(np.uint32).tobytes()).hexdigest() for b in bufs}
            assert ent["argb_sha"] in shas
            if n >= nbuf:
                assert shas == {ent["argb_sha"]}, (key, nbuf, n)
        assert s.cam.device_error(reset=True) == 0
    with pytest.raises(_lib.RtError):
        R.FrameLoop(s.cam, bufs, mode=0, render_stream=st.cuda_stream, inflight=_lib.RT_LOOP_MULTIFRAME,
                    xforms=np.stack([np.eye(3, 4, dtype=np.float32).reshape(12)] * 2)).run(4)


@pytest.mark.parametrize("order", [0, 4, 5])
@pytest.mark.parametrize("key", ["dragon_960x540_m0", "knot_1920x1080_m0"])
def test_multiframe_xcd_orders(key, order):
    """Round 6 (verdict r05 item 5): the XCD-mapped tile orders pad every
    frame of a multi-frame launch to a multiple of 8 blocks (the padding
    blocks exit); every buffer set still holds the oracle's frame, and the
    cost-ordered ones (4, 5) take their cost samples from single-frame
    launches first."""
    import hashlib
    import torch
    from cpp_cuda_raytracer_dev_amd import _lib
    ent = H.frame_hashes()[key]
    if not H.mesh_matches(ent):
        pytest.skip("stand-in mesh bits differ on this host")
    w, h = ent["w"], ent["h"]
    s = H.GpuScene(ent["scene"], w, h, tile_order=order)
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(device=dev)
    bufs = [torch.full((w * h,), 0x7BADBEEF, dtype=torch.int32, device=dev) for _ in range(3)]
    loop = R.FrameLoop(s.cam, bufs, mode=0, render_stream=st.cuda_stream, event_every=1,
                       inflight=_lib.RT_LOOP_MULTIFRAME)
    for n in (40, 200):
        for b in bufs:
            b.fill_(0x7BADBEEF)
        torch.cuda.synchronize()
        loop.run(n)
        torch.cuda.synchronize()
        shas = {hashlib.sha256(b.cpu().numpy().view(np.uint32).tobytes()).hexdigest() for b in bufs}
        assert shas == {ent["argb_sha"]}, (key, order, n)
    assert s.cam.device_error(reset=True) == 0
    s.close()


def test_multiframe_alternating_loops_kept_order():
    """a small frame whose rays-per-wave rule differs between
    multi-frame launches (32) and the per-frame loop (16) switches tilings on
    every rt_run_frames call; each switch starts from the cost order last
    measured for that tiling (rt_api.cpp restore_order).  Every frame of
    every call is still the oracle's (committed hash)."""
    import hashlib
    import torch
    from cpp_cuda_raytracer_dev_amd import _lib
    ent = H.frame_hashes()["dragon_960x540_m0"]
    if not H.mesh_matches(ent):
        pytest.skip("stand-in mesh bits differ on this host")
    w, h = ent["w"], ent["h"]
    s = H.GpuScene(ent["scene"], w, h)
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(device=dev)
    bufs = [torch.full((w * h,), 0x7BADBEEF, dtype=torch.int32, device=dev) for _ in range(2)]
    mf = R.FrameLoop(s.cam, bufs, mode=0, render_stream=st.cuda_stream, event_every=1,
                     inflight=_lib.RT_LOOP_MULTIFRAME)
    lanes = R.FrameLoop(s.cam, bufs, mode=0, render_stream=st.cuda_stream, event_every=8, inflight=2)
    used = set()
    restores = []
    for i in range(6):
        loop = mf if i % 2 == 0 else lanes
        for b in bufs:
            b.fill_(0x7BADBEEF)
        torch.cuda.synchronize()
        loop.run(60)
        torch.cuda.synchronize()
        used.add(s.cam.get_option(_lib.RT_OPT_RAYS_USED))
        restores.append(s.cam.get_option(_lib.RT_OPT_ORDER_RESTORES))
        shas = {hashlib.sha256(b.cpu().numpy().view(np.uint32).tobytes()).hexdigest() for b in bufs}
        assert shas == {ent["argb_sha"]}, (i, s.cam.get_option(_lib.RT_OPT_RAYS_USED))
    assert used == {16, 32}
    # the kept orders are really restored.  The first call of
    # each tiling measures its order (60 frames hold several cost samples);
    # from the third call on, every switch restarts from the kept one.
    assert restores[0] == restores[1] == 0, restores
    assert all(restores[i] == restores[i - 1] + 1 for i in range(2, 6)), restores
    assert s.cam.device_error(reset=True) == 0
    s.close()


# kFast walks (rt_kernels_impl.h fast_slot / order_node<kFast>): the float
# entry test and the float ordering thresholds must give the reference's
# frame, its visit counts included, wherever rt_api.cpp fast_proof admits
# the frame.  Each pose renders with the proof's walks and with debug bit
# 2048 (the double-promoted forms) and the two must agree bit for bit; the
# default view is also checked against the oracle.
FAST_POSES = [None,  # the default view (eye at z = -1, looking +z)
              dict(pos=(0.9, 0.35, 0.2), look_at=(0.0, 0.1, 0.0)),     # from the side (proof along x)
              dict(pos=(0.05, 1.2, 0.01), look_at=(0.0, 0.1, 0.0)),    # from above (along y)
              dict(pos=(-0.3, 0.0, 0.6), look_at=(0.0, 0.12, 0.0)),    # from behind, below
              dict(pos=(0.0, 0.1, -0.25), look_at=(0.0, 0.1, 0.0))]    # close in front (large field)


def _fast_pair(scene, w, h, kw=None, xf=None, shadow=False, rays=None):
    """Renders a frame with the proof's walks and with debug bit 2048 (the
    double-promoted forms), counted and timed; returns both (argb, hit,
    counters, RT_OPT_FAST_USED) after checking counted == timed."""
    from cpp_cuda_raytracer_dev_amd import _lib
    outs = []
    for debug in (0, 2048):
        s = H.GpuScene(scene, w, h, cam_kw=kw, kernel=3, debug=debug, rays=rays)
        try:
            argb, hit, cnt = s.render(0, xform=xf, count=True, shadow=shadow)
            used = s.cam.get_option(_lib.RT_OPT_FAST_USED)
            argb2, hit2, _ = s.render(0, xform=xf, shadow=shadow)  # the timed (uncounted) instance
        finally:
            s.close()
        _assert_same((argb2, hit2), (argb, hit), f"{scene} debug {debug} counted vs timed")
        outs.append((argb, hit, [int(x) for x in cnt], used))
    assert outs[1][3] == 0
    _assert_same(outs[0][:2], outs[1][:2], f"{scene} fast vs double forms")
    assert outs[0][2] == outs[1][2], (outs[0][2], outs[1][2])
    return outs


@pytest.mark.parametrize("shadow", [False, True])
@pytest.mark.parametrize("pose", range(len(FAST_POSES)))
@pytest.mark.parametrize("scene,w,h", [("tester", 320, 180), ("rabbit_70k", 480, 270), ("dragon", 480, 270)])
def test_fast_walk_same_frame(scene, w, h, pose, shadow):
    """Round 6: the shadow walks too (xfast_slot under the light's proof,
    verdict r05 item 2); tester.ply's light lies inside its root box, so its
    shadow frames keep the double forms (and show no shadows)."""
    kw = FAST_POSES[pose]
    outs = _fast_pair(scene, w, h, kw=kw, shadow=shadow)
    if kw is None:
        assert outs[0][3] & 1, "the default view proves the float entry test"
        if shadow and scene != "tester":
            assert outs[0][3] & 2, "the light (2, 2, 2) lies beyond the root box: the shadow walks' proof"
        oargb, ohit, ocnt = H.oracle_render(scene, w, h, 0, shadow=shadow)
        _assert_same(outs[0][:2], (oargb, ohit), f"{scene} fast vs oracle")
        if not shadow:
            _counters_match(outs[0][2], ocnt, 3)
    if shadow and scene == "tester" and kw is None:
        assert not outs[0][3] & 2  # (the light moves with the camera: other poses may prove it)


# Object transforms (verdict r05 item 3: the reference's keyboard path,
# TD/WinMain.cpp:186-209 -> TD/Camera.cu:254-335): a rotation keeps the
# untranslated walk (kFast slots under the rotated proof), an offset takes
# the translated walk's xfast_slot; both must equal the double forms.
FAST_XFORMS = [_rot_y(17.0), _rot_y(0.0, (0.01, -0.005, 0.02)), _rot_y(-9.0, (0.0, 0.01, 0.0)),
               _rot_y(31.0, (0.05, 0.02, 0.3)), _rot_y(-52.0, (-0.03, 0.0, -0.2))]


@pytest.mark.parametrize("shadow", [False, True])
@pytest.mark.parametrize("xi", range(len(FAST_XFORMS)))
@pytest.mark.parametrize("scene", ["rabbit_70k", "dragon"])
def test_fast_walk_transforms(scene, xi, shadow):
    xf = FAST_XFORMS[xi]
    outs = _fast_pair(scene, 480, 270, xf=xf, shadow=shadow)
    assert outs[0][3] & 5 == 5, f"the transformed frame proves the float entry test ({outs[0][3]})"
    if shadow:
        assert outs[0][3] & 2
    if xi < 2:
        oargb, ohit, _ = H.oracle_render(scene, 480, 270, 0, xform=xf, shadow=shadow)
        assert (ohit >= 0).sum() > 100
        _assert_same(outs[0][:2], (oargb, ohit), f"{scene} xform {xi} fast vs oracle")


@pytest.mark.parametrize("rays", [8, 16, 32])
def test_fast_walk_transform_rays(rays):
    """Every unit width's translated and shadow fast walks (the 8-, 16- and
    32-ray instances), against the double forms and the oracle."""
    xf = FAST_XFORMS[2]
    outs = _fast_pair("dragon", 480, 270, xf=xf, shadow=True, rays=rays)
    assert outs[0][3] & 7 == 7
    oargb, ohit, _ = H.oracle_render("dragon", 480, 270, 0, xform=xf, shadow=True)
    _assert_same(outs[0][:2], (oargb, ohit), f"dragon rays {rays} fast vs oracle")


def test_fast_walk_refused_inside_box():
    """An eye inside the root box on every axis: no axis proves the entry
    test, so the walks keep the double-promoted forms."""
    from cpp_cuda_raytracer_dev_amd import _lib
    s = H.GpuScene("dragon", 320, 180, cam_kw=dict(pos=(0.0, 0.12, 0.0), look_at=(0.0, 0.12, 1.0)), kernel=3)
    try:
        argb, hit, _ = s.render(0)
        assert s.cam.get_option(_lib.RT_OPT_FAST_USED) == 0
    finally:
        s.close()
    oargb, ohit, _ = H.oracle_render("dragon", 320, 180, 0,
                                     cam_kw=dict(pos=(0.0, 0.12, 0.0), look_at=(0.0, 0.12, 1.0)))
    _assert_same((argb, hit), (oargb, ohit), "dragon inside the root box vs oracle")


def test_rcp_newton_exhaustive():
    """rcp_nr (rt_kernels_impl.h: v_rcp_f32 and one fused Newton step), which
    kFast walks use for 1/r and the leaf test's 1/f, equals the correctly
    rounded 1.0f / x for every float of magnitude in [2^-126, 2^126), both
    signs (4.23e9 values; tools/check_rcp.hip, built by build.py)."""
    import json
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "check_rcp")
    if not os.path.exists(exe):
        pytest.fail("tools/check_rcp is not built (python -m cpp_cuda_raytracer_dev_amd.build)")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=100)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0 and out["bad"] == 0 and out["checked"] == 2 * 252 * (1 << 23), out


@pytest.mark.parametrize("scene", ["dragon", "rabbit_70k"])
def test_fast_walk_tiny_s1_fixup(scene):
    """kFast walks take s1 itself as the reference's (float)((double)s1 +
    1e-16) except on records where that sum rounds off s1 (k_cam_nodes'
    tiny-s1 flag), which take the double form.  A camera whose x (or y) lies
    exactly on an interior node's s1 makes that node's camera-relative s1 a
    zero (0 + 1e-16 rounds to 1e-16, not 0), so the camera's records carry
    the flag and the fix-up runs; the frame, hit buffer and counters equal
    the double-form walk's (debug bit 2048) and the oracle's."""
    from cpp_cuda_raytracer_dev_amd import _lib
    nodes = H.product_tree(scene)
    interior = np.flatnonzero((nodes["is_leaf"] == 0) & (nodes["cut_flag"] % 3 != 2))
    k = int(interior[min(3, len(interior) - 1)])
    axis = int(nodes["cut_flag"][k]) % 3
    pos = [0.0, 0.1, -1.0]
    pos[axis] = float(nodes["s1"][k])
    look = [pos[0], pos[1], 0.0]
    kw = dict(pos=tuple(pos), look_at=tuple(look))
    w, h = 320, 180
    outs = []
    for debug in (0, 2048):
        s = H.GpuScene(scene, w, h, cam_kw=kw, kernel=3, debug=debug)
        try:
            argb, hit, cnt = s.render(0, count=True)
            used = s.cam.get_option(_lib.RT_OPT_FAST_USED)
            argb2, hit2, _ = s.render(0)
        finally:
            s.close()
        _assert_same((argb2, hit2), (argb, hit), f"{scene} tiny-s1 debug {debug} counted vs timed")
        outs.append((argb, hit, [int(x) for x in cnt], used))
    assert outs[0][3] == 1, outs[0][3]  # kFast walks (with the fix-up: the relative s1 of node k is 0)
    assert np.float32(nodes["s1"][k]) - np.float32(pos[axis]) == 0.0
    assert outs[1][3] == 0
    _assert_same(outs[0][:2], outs[1][:2], f"{scene} tiny-s1 fast vs double forms")
    assert outs[0][2] == outs[1][2]
    oargb, ohit, ocnt = H.oracle_render(scene, w, h, 0, cam_kw=kw)
    _assert_same(outs[0][:2], (oargb, ohit), f"{scene} tiny-s1 fast vs oracle")
    _counters_match(outs[0][2], ocnt, 3)
