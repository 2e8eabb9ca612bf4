#!/usr/bin/env python3
"""Benchmark: frames/s and Mray/s at 1920x1080 on the dragon (stand-in),
KD traversal, 1..N MI355X GPUs (BASELINE.json metric; configs C3/C4).

The default workload is the torus-knot stand-in (`--scene knot`): the
dragon's 871,414 triangles in the dragon's box as a noise-displaced (5, 12)
torus-knot tube, strands in front of strands, ~1.9x the interior visits per
covered ray of the displaced-sphere blob (`--scene dragon`), which stays as a
secondary line.  SURVEY.md §8d suggests the knot as the dragon stand-in.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

A step is one frame: bg fill -> primary rays -> KD traversal -> Moller-
Trumbore -> Phong into the u32 frame (one fused kernel), plus, for N > 1,
the RCCL gather to rank 0 of every rank's screen bands (the part of them
not provably background) and the frame assembly kernel there, pipelined
with the next frame's render.  Frames are fixed-size (1920x1080), so N > 1 is strong
scaling.  The scene is a seeded synthetic stand-in for
dragon_vrip_mod.ply (missing from the reference; 871,414 triangles).
Rank 0 prints one JSON line.

The other BASELINE configs are selected with flags:
    C1  --cpu-only --scene tester --width 320 --height 180   (CPU path, no GPU)
    C2  --scene rabbit_70k --width 960 --height 540 --mode 1  (flat list, VALU roofline)
    C3  --width 960 --height 540
    C5  --scene happy --width 3840 --height 2160 --shadow
and README.md:19's high-coverage view with --view fill.

After the timed frames every line carries `device_err` (the camera's device
error word; the run exits non-zero when it is set) and, at N = 1, a
`frame_check`: the last timed frame against the oracle's committed full-frame
hash (tests/golden/frame_hashes.json), or against an oracle render on this
host when no hash matches.  With multi-frame launches as the headline (the
default at N = 1 for a static KD frame), the line also carries
`per_frame_loop`: --second-frames frames of the per-frame loop (two frames in
flight on the library's render lanes), timed after the headline with their own
settle and frame check -- the rate a loop with new input every frame sees.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/sec + Mray/s at 1920×1080, Stanford dragon 800k tris, 1/2/4/8 GPU"
W, H = 1920, 1080
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# FP32 vector peak without FMA: the spec's 157.3 TFLOP/s (MI355X_MICROARCH.md)
# counts a packed FMA as 4 flops per lane; with contraction off every flop is
# its own operation, so the ceiling is 157.3 / 2 = 78.6 TFLOP/s with packed
# v_pk_mul_f32 / v_pk_add_f32 and 39.3 unpacked.  tools/ubench_pk.hip measured
# 64.8 (packed) and 34.6 (unpacked) T mul+add/s: 82 % and 88 % of those.
VALU_PEAK_TFLOPS, VALU_PEAK_UNPACKED_TFLOPS = 78.6, 39.3
# 28 FP32 flops + one correctly rounded divide per flat test
FLOPS_PER_TEST = 28
HASHES = os.path.join(ROOT, "tests", "golden", "frame_hashes.json")
# bytes per interior visit, leaf visit, accepted hit, pixel
B_INT, B_LEAF, B_HIT, B_PIX = 36, 40, 24, 4


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs (ranks); N > 1 without torch.distributed.run starts its own N rank processes")
    ap.add_argument("--launch-dry-run", action="store_true",
                    help="with --gpus N: start the N rank processes, each of which prints its rank environment "
                         "as JSON and exits without touching a GPU (tests the launcher on CPU)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--scene", default="knot", choices=["dragon", "happy", "rabbit_70k", "tester", "big", "knot"],
                    help="knot (default) / dragon / happy: seeded stand-ins for the missing meshes (knot: the dragon's "
                         "count and box as a torus-knot tube, ~2x the blob's traversal work; dragon: a displaced-sphere "
                         "blob; big: a 3.1M-triangle one); rabbit_70k / tester: the reference's own meshes")
    ap.add_argument("--view", default="default", choices=["default", "fill"],
                    help="default: WinMain's camera; fill: the object over >= 90%% of the pixels (README.md:19)")
    ap.add_argument("--cpu-only", action="store_true",
                    help="config C1: the CPU path only (the oracle), no GPU; value = its frames/s")
    ap.add_argument("--width", type=int, default=W)
    ap.add_argument("--height", type=int, default=H)
    ap.add_argument("--mode", type=int, default=0, help="0 KD, 1 flat list")
    ap.add_argument("--collective", default="rccl", choices=["rccl", "gather", "allgather"],
                    help="N>1 frame gather: rccl = the library's own RCCL send/recv + unpack (rt_comm_*, "
                         "pipelined); gather / allgather = torch.distributed collectives, one frame at a time")
    ap.add_argument("--rehearse-gather", action="store_true",
                    help="one process: run the N>1 frame loop (process group, gather, frame check) with one rank, "
                         "to rehearse the multi-GPU path on a one-GPU machine; not a bench line")
    ap.add_argument("--loop", default="native", choices=["native", "python"],
                    help="frame loop: native = rt_run_frames (C++, the render + RCCL gather enqueued per frame "
                         "without Python), python = the same calls from Python (torch collectives, --animate)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="native loop: 0 = automatic (multi-frame launches for a static KD scene without shadow rays "
                         "at one GPU, else 2), -1 = multi-frame launches (RT_LOOP_MULTIFRAME: one grid of many frames' "
                         "blocks, frame-major; static scene, N = 1), else frames in flight on the library's render "
                         "lanes (rt_frame_loop.inflight; "
                         "1 = one frame at a time).  The roofline's kernel time comes from a separate pass of "
                         "solo frames (one in flight), since overlapped launches share the GPU")
    ap.add_argument("--solo-frames", type=int, default=200,
                    help="inflight > 1: solo frames (one in flight, every one bracketed by events) before the "
                         "timed region, for the roofline's kernel time")
    ap.add_argument("--solo-when", default="before", choices=["before", "after"],
                    help="solo frames (the roofline's kernel time) run just before the warm-up-to-timed handover, "
                         "or after the timed frames")
    ap.add_argument("--second-frames", type=int, default=1000,
                    help="with multi-frame launches as the headline: also time this many frames of the per-frame "
                         "loop (two frames in flight on the library's render lanes) after it and report them as "
                         "the line's per_frame_loop object (0 = off)")
    ap.add_argument("--settle-ms", type=float, default=40.0,
                    help="untimed frames of the timed loop itself for about this much time right before the timed "
                         "region (a moving object: one pass over the timed poses, native loop only; 0: none)")
    ap.add_argument("--pipeline", type=int, default=2,
                    help="rccl: buffer sets in flight (frame i+1 renders while frame i is gathered)")
    ap.add_argument("--kernel", type=int, default=3,
                    help="KD kernel: 2 per-lane DFS in the reference's order, 3 wave-cooperative item pool")
    ap.add_argument("--tile-order", type=int, default=3,
                    help="0 XCD-contiguous, 1 natural, 2 centre-out, 3 by the cost an earlier frame measured")
    ap.add_argument("--rays", type=int, default=0,
                    help="kernel 3: pixels per wave (32, 16, 8; 0 = the library's automatic choice)")
    ap.add_argument("--items", type=int, default=2, help="kernel 3: items each lane pops per iteration (1, 2; 65..128: two only when the pool holds that many)")
    ap.add_argument("--order", type=int, default=-1,
                    help="interior record order: 0 BFS, 1 DFS preorder, 2 treelets (-1: the library default)")
    ap.add_argument("--treelet", type=int, default=0, help="treelet height for --order 2 (0: library default)")
    ap.add_argument("--flat", type=int, default=-1,
                    help="flat-list kernel form: 9 one pass, 12 the list in 16 chunks (-1: the library default, 12)")
    ap.add_argument("--coarse", type=int, default=8,
                    help="kernel 3: 8x8 groups per wave outside the root box's screen rectangle (0 = off)")
    ap.add_argument("--event-every", type=int, default=0,
                    help="bracket every Nth timed frame with HIP events for the kernel time (each pair costs "
                         "~9 us of queue time, so N > 1 keeps the frame rate close to the uninstrumented one); "
                         "0 = every 8th (every frame with --inflight 1 at one GPU)")
    ap.add_argument("--debug-bits", type=int, default=0,
                    help="diagnostics: extra RT_OPT_DEBUG bits for the timed camera (A/B builds of host policies)")
    ap.add_argument("--side-coarse", action="store_true",
                    help="kernel 3: run the coarse kernel beside the fine one on a side stream (default: before it)")
    ap.add_argument("--deliver", action="store_true",
                    help="N=1: also time frames delivered to pinned host memory (render + async D2H, double "
                         "buffered); reported in a 'delivery' object, never as value")
    ap.add_argument("--shadow-order", type=int, default=-1,
                    help="kernel 3 any-hit push order 0..3, -1 = timed choice (default)")
    ap.add_argument("--animate", default="",
                    help="held keys per frame, cycled: letters R W S Q E T, '+' joins keys held together, '.' is "
                         "a tick with none; one input tick (TD/WinMain.cpp:186-209) before each frame, timed")
    ap.add_argument("--shadow", action="store_true",
                    help="one shadow ray per hit (config C5: --scene happy --width 3840 --height 2160 --shadow)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="CPU baseline sample length, for each of the 1-thread and all-thread runs")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0: OMP_NUM_THREADS, else the CPUs this process may use)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def build_scene(name):
    """(points9, leafs, nodes, timings): read_ply's face assembly and the KD
    build (a11) on this host, the build timed with all threads and one."""
    from cpp_cuda_raytracer_dev_amd import raytracer as R, scenes
    v, arity, idx = scenes.mesh_arrays(name)
    pts, n, leafs = R.assemble_mesh(v, scenes.faces_of(arity, idx))
    t0 = time.perf_counter()
    nodes = R.kd_build(leafs)
    t1 = time.perf_counter()
    R.kd_build(leafs, nthreads=1)
    t2 = time.perf_counter()
    return pts, leafs, nodes, {"kd_build_s": round(t1 - t0, 4), "kd_build_s_1thread": round(t2 - t1, 4)}


def cpu_quota():
    """CPUs' worth of time the cgroup grants this process (cgroup v2 cpu.max or
    v1 cfs_quota/period), or None when unlimited / unknown."""
    import math
    try:
        with open("/sys/fs/cgroup/cpu.max") as fp:
            q, per = fp.read().split()[:2]
            return None if q == "max" else max(1, math.ceil(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else max(1, math.ceil(q / per))
    except (OSError, ValueError):
        return None


def cpu_threads(requested: int) -> int:
    """Threads of the CPU baseline: every CPU this process may use -- its
    affinity mask, capped by its cgroup CPU quota (threads beyond the quota
    only time-slice).  OMP_NUM_THREADS is not consulted."""
    if requested > 0:
        return requested
    n = len(os.sched_getaffinity(0))
    q = cpu_quota()
    return min(n, q) if q else n


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fp:
            for line in fp:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _lib_mod():
    from cpp_cuda_raytracer_dev_amd import _lib
    return _lib


def data_label(scene: str) -> str:
    from cpp_cuda_raytracer_dev_amd import scenes
    return "synthetic" if scene in scenes.STANDINS else f"{scene}.ply from the reference (TD/), parsed with strtof"


def frame_key(scene, w, h, mode, shadow, view):
    return f"{scene}_{w}x{h}_m{mode}" + ("_shadow" if shadow else "") + ("" if view == "default" else f"_{view}")


def reference_frame(scene, w, h, mode, shadow, view):
    """The committed oracle entry for this frame (tests/golden/frame_hashes.json)
    when its mesh bytes equal this host's, else None."""
    from cpp_cuda_raytracer_dev_amd import scenes
    try:
        with open(HASHES) as fp:
            ent = json.load(fp)["frames"].get(frame_key(scene, w, h, mode, shadow, view))
    except (OSError, ValueError, KeyError):
        return None
    if ent is None or ent.get("mesh_sha") != scenes.mesh_sha(scene):
        return None
    return ent


def frame_check_n1(argb: np.ndarray, pts, nodes, cam_kw, a, xform=None):
    """The last timed frame against the oracle: its committed full-frame hash,
    or (no hash for this frame / mesh, or a moved object) an oracle render
    here (KD mode)."""
    import hashlib
    got = hashlib.sha256(np.ascontiguousarray(argb).tobytes()).hexdigest()
    ent = None if a.animate else reference_frame(a.scene, a.width, a.height, a.mode, a.shadow, a.view)
    if ent is not None:
        return {"matches_oracle": got == ent["argb_sha"], "method": "sha256 vs tests/golden/frame_hashes.json "
                f"[{frame_key(a.scene, a.width, a.height, a.mode, a.shadow, a.view)}]"}
    if a.mode != 0:
        return {"matches_oracle": None, "method": "no committed hash; the flat oracle is too slow to run here"}
    from oracle import _oracle as O
    on = np.zeros(len(nodes), O.NODE_DTYPE)
    for k in nodes.dtype.names:
        on[k] = nodes[k]
    s = O.Scene(pts, O.default_rad(len(pts)), on, O.camera(a.width, a.height, **cam_kw))
    ref, _, _ = s.render(0, xform=xform, nthreads=cpu_threads(a.cpu_threads), want_hit=False, shadow=a.shadow)
    s.close()
    return {"matches_oracle": bool(np.array_equal(ref, argb)), "method": "oracle render on this host"}


def _oracle_fps(s, mode, rows, h, seconds, threads, shadow):
    frames, t0 = 0, time.perf_counter()
    while True:
        s.render(mode, rows=rows, nthreads=threads, want_hit=False, shadow=shadow)
        frames += 1
        if time.perf_counter() - t0 >= seconds and frames >= 2:
            break
    dt = time.perf_counter() - t0
    return frames * (rows[1] - rows[0]) / h / dt, frames, dt


def cpu_baseline(pts, nodes, w, h, seconds, threads, mode, shadow=False, rays_per_frame=None, cam_kw=None,
                 build_times=None):
    """The oracle (C restatement, gcc -O3 -ffp-contract=off, OpenMP over rows)
    on the same frame, repeated for ~`seconds` with all `threads` and with
    one.  The reference has no CPU intersect path, so this
    restatement is the CPU baseline (kind "port").  Test infrastructure: the
    checker, timed beside the GPU; never part of the product path."""
    from oracle import _oracle as O
    on = np.zeros(len(nodes), O.NODE_DTYPE)
    for k in nodes.dtype.names:
        on[k] = nodes[k]
    s = O.Scene(pts, O.default_rad(len(pts)), on if mode == 0 else None, O.camera(w, h, **(cam_kw or {})))
    rows = (0, h)
    if mode == 1:  # flat list is O(npix*ntri): sample a band of rows through the object
        rows = (h // 2 - 4, h // 2 + 4)
    fps, frames, dt = _oracle_fps(s, mode, rows, h, seconds, threads, shadow)
    rows1 = rows if mode == 1 else (h // 2 - h // 16, h // 2 + h // 16)  # one thread: the middle eighth
    fps1, frames1, dt1 = _oracle_fps(s, mode, rows1, h, seconds, 1, shadow)
    extra = {}
    allowed = len(os.sched_getaffinity(0))
    if threads < allowed:
        # the whole affinity mask too (beyond the quota it only time-slices)
        fa, _, _ = _oracle_fps(s, mode, rows, h, seconds / 2, allowed, shadow)
        extra = {"value_cpus_allowed_threads": round(fa, 3), "cpus_allowed_threads": allowed}
    if threads != 16 and allowed >= 16:
        f16, _, _ = _oracle_fps(s, mode, rows, h, seconds / 2, 16, shadow)
        extra["value_16threads"] = round(f16, 3)
    s.close()
    rpf = rays_per_frame or w * h
    out = {"value": round(fps, 3), "unit": "frames/s", "cores": threads, "kind": "port",
           "mray_per_s": round(fps * rpf / 1e6, 3),
           "value_1thread": round(fps1, 3), "mray_per_s_1thread": round(fps1 * rpf / 1e6, 3), **extra,
           "nproc": os.cpu_count(), "cpus_allowed": allowed, "cpu_quota_cpus": cpu_quota(),
           "threads_rule": "every CPU of the affinity mask, capped by the cgroup CPU quota",
           "cpu_model": cpu_model(),
           "sample": f"{frames} x rows {rows[0]}-{rows[1]} of the same {w}x{h} frame with {threads} threads "
                     f"({dt:.1f} s), {frames1} x rows {rows1[0]}-{rows1[1]} with 1 thread ({dt1:.1f} s); "
                     "oracle/oracle.c (gcc -O3 -ffp-contract=off, OpenMP over rows)"}
    if build_times:
        out["kd_build"] = {**build_times, "what": "rt_kd_build (a11, TD/Trixel.h:135-473) on this host, all "
                                                  "threads / 1 thread; rt_kd_build_gpu on the GPU (host in/out)"}
    return out


def cpu_only(a):
    """Config C1: the CPU path alone (no GPU): the oracle's full frames."""
    from cpp_cuda_raytracer_dev_amd import scenes
    from oracle import _oracle as O
    import hashlib
    w, h = a.width, a.height
    pts, leafs, nodes, bt = build_scene(a.scene)
    on = np.zeros(len(nodes), O.NODE_DTYPE)
    for k in nodes.dtype.names:
        on[k] = nodes[k]
    cam_kw = scenes.view(a.scene, a.view)
    s = O.Scene(pts, O.default_rad(len(pts)), on if a.mode == 0 else None, O.camera(w, h, **cam_kw))
    threads = cpu_threads(a.cpu_threads)
    argb, hit, cnt = s.render(a.mode, nthreads=threads, shadow=a.shadow)
    fps, frames, dt = _oracle_fps(s, a.mode, (0, h), h, a.cpu_seconds, threads, a.shadow)
    fps1, frames1, dt1 = _oracle_fps(s, a.mode, (0, h), h, a.cpu_seconds, 1, a.shadow)
    s.close()
    ent = reference_frame(a.scene, w, h, a.mode, a.shadow, a.view)
    got = hashlib.sha256(argb.tobytes()).hexdigest()
    rpf = w * h + (int((hit >= 0).sum()) if a.shadow else 0)
    res = {
        "metric": METRIC, "value": round(fps, 2), "unit": "frames/s", "mray_per_s": round(fps * rpf / 1e6, 3),
        "n_gpus": 0, "steps": frames, "warmup": 1, "ms_per_step": round(1e3 * dt / frames, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": data_label(a.scene),
        "config": {"workload": f"{a.scene} {w}x{h}, CPU-only intersect path ({'KD traversal' if a.mode == 0 else 'flat list'}"
                               " + Phong, u32 frame), config C1",
                   "scene": f"{a.scene} ({len(pts)} triangles)", "resolution": [w, h], "view": a.view,
                   "coverage": round(float((hit >= 0).mean()), 4), "parallelism": f"OpenMP x{threads}"},
        "roofline": None,
        "frame_check": {"matches_oracle": (got == ent["argb_sha"]) if ent else None,
                        "method": "sha256 vs tests/golden/frame_hashes.json" if ent else "no committed hash"},
        "cpu_baseline": {"value": round(fps, 3), "unit": "frames/s", "cores": threads, "kind": "port",
                         "value_1thread": round(fps1, 3), "nproc": os.cpu_count(),
                         "cpus_allowed": len(os.sched_getaffinity(0)), "cpu_model": cpu_model(),
                         "kd_build": bt,
                         "sample": f"{frames} full frames with {threads} threads ({dt:.1f} s), {frames1} with 1 thread "
                                   f"({dt1:.1f} s); oracle/oracle.c (gcc -O3 -ffp-contract=off)"},
        "note": "C1 is the CPU path (BASELINE.json configs[0]): the reference has no CPU intersect path, so this is "
                "the build's C restatement (oracle/oracle.c); no GPU kernel runs, so there is no roofline",
    }
    print(json.dumps(res), flush=True)
    return 0 if res["frame_check"]["matches_oracle"] is not False else 1


def delivery(cam, R, torch, dev, w, h, xf, mode, sflag, steps, warmup):
    """Frames delivered to the host: frame i renders
    into device buffer i % 2 on the render stream while frame i - 1's D2H into
    pinned host memory runs on a copy stream.  Returns frames/s and the D2H
    rate; PCIe-inclusive, so reported beside `value`, never as it."""
    npix = w * h
    outs = [torch.zeros(npix, dtype=torch.int32, device=dev) for _ in range(2)]
    pf = R.PinnedFrames(npix, 2)
    rs, cs = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    rendered = [torch.cuda.Event() for _ in range(2)]
    copied = [torch.cuda.Event() for _ in range(2)]

    def one(i):
        k = i % 2
        rs.wait_event(copied[k])  # the copy of frame i - 2 has left buffer k
        cam.render_into(outs[k], xform=xf, mode=mode, flags=sflag, stream=rs.cuda_stream)
        rendered[k].record(rs)
        cs.wait_event(rendered[k])
        pf.copy_async(k, dev.index, outs[k], stream=cs.cuda_stream)
        copied[k].record(cs)

    for k in range(2):
        copied[k].record(cs)
    for i in range(warmup):
        one(i)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(steps):
        one(i)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    ok = bool((pf.frames[(steps - 1) % 2] == outs[(steps - 1) % 2].cpu().numpy().view(np.uint32)).all())
    pf.close()
    return {"frames_per_s": round(steps / dt, 2), "d2h_gb_per_s": round(steps * npix * 4 / dt / 1e9, 2),
            "frame_bytes": npix * 4, "steps": steps, "host_frame_matches_device": ok,
            "method": "render on one stream, D2H to pinned host memory on another, 2 buffers"}


def key_masks(spec: str) -> list:
    """"R+W.Q" -> [R|W, 0, Q] (bits of raytracer.KEY_*), as tools/rt_headless reads it."""
    from cpp_cuda_raytracer_dev_amd import raytracer as R
    bits = {"R": R.KEY_R, "W": R.KEY_W, "S": R.KEY_S, "Q": R.KEY_Q, "E": R.KEY_E, "T": R.KEY_T, ".": 0}
    out = []
    k = 0
    while k < len(spec):
        m = 0
        while True:
            c = spec[k]
            if c not in bits:
                raise ValueError(f"--animate: unknown key {c!r}")
            m |= bits[c]
            k += 1
            if k < len(spec) and spec[k] == "+":
                k += 1
                continue
            break
        out.append(m)
    return out


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpu_count():
    """The GPUs a rank process could use, counted without torch, amdsmi or
    HIP (torch.cuda.device_count() falls back to
    hipGetDeviceCount, which initialises HIP, whenever amdsmi fails): the
    KFD topology's nodes with SIMDs (a CPU node has simd_count 0), in node
    order, then narrowed by ROCR_VISIBLE_DEVICES and HIP_VISIBLE_DEVICES
    (CUDA_VISIBLE_DEVICES when HIP's is unset), each a comma list of indices
    into the devices the previous filter left.  UUID entries count as one
    device each.  None when the topology cannot be read (the ROCm runtime
    enumerates GPUs from the same files, so a host whose runtime works has
    it).  RT_KFD_TOPOLOGY names another topology directory (tests)."""
    root = os.environ.get("RT_KFD_TOPOLOGY", "/sys/class/kfd/kfd/topology/nodes")
    try:
        names = sorted((d for d in os.listdir(root) if d.isdigit()), key=int)
    except OSError:
        return None
    n = 0
    for d in names:
        try:
            with open(os.path.join(root, d, "properties")) as fp:
                props = dict(line.split(None, 1) for line in fp if len(line.split(None, 1)) == 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0").strip() or 0) > 0:
            n += 1

    def narrow(count: int, spec) -> int:
        if spec is None:
            return count
        keep = 0
        for tok in (t.strip() for t in spec.split(",")):
            if not tok:
                break
            if tok.isdigit():
                if int(tok) >= count:
                    break  # the runtimes stop at the first invalid index
                keep += 1
            else:
                keep += 1  # a UUID names one device
        return min(keep, count)

    n = narrow(n, os.environ.get("ROCR_VISIBLE_DEVICES"))
    hip = os.environ.get("HIP_VISIBLE_DEVICES")
    return narrow(n, hip if hip is not None else os.environ.get("CUDA_VISIBLE_DEVICES"))


def launch_ranks(a) -> int:
    """`--gpus N` (N > 1) without torch.distributed.run (WORLD_SIZE unset):
    start N fresh rank processes of this script with RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR (127.0.0.1) / MASTER_PORT set, one per GPU, and
    wait for them.  This process never touches a GPU,
    nor loads torch or the HIP runtime: it counts the visible devices from
    the KFD topology (visible_gpu_count) and fails fast when there are fewer
    than N.  Rank 0 prints the JSON line.  When a rank fails the others get
    60 s to finish, then are killed (by PID); the first failing rank's exit
    code is returned.  RT_BENCH_LAUNCH_MAPS (tests) names a file the parent
    copies its /proc/self/maps into just before it starts the ranks."""
    import subprocess
    n = a.gpus
    have = visible_gpu_count()
    if have is None:
        print("bench.py: no KFD topology to count GPUs from; starting the ranks unchecked", file=sys.stderr, flush=True)
    elif have < n:
        print(f"bench.py: --gpus {n} but only {have} GPU(s) visible", file=sys.stderr, flush=True)
        return 2
    if os.environ.get("RT_BENCH_LAUNCH_MAPS"):
        with open("/proc/self/maps") as src, open(os.environ["RT_BENCH_LAUNCH_MAPS"], "w") as dst:
            dst.write(src.read())
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RT_BENCH_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc, deadline = 0, None
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad and not rc:
            rc = bad[0][1]
            print(f"bench.py: rank {bad[0][0]} exited {rc}", file=sys.stderr, flush=True)
            deadline = time.monotonic() + 60.0
        if all(c is not None for c in codes):
            break
        if deadline is not None and time.monotonic() > deadline:
            for p in procs:
                if p.poll() is None:
                    p.kill()
            for p in procs:
                p.wait()
            break
        time.sleep(0.1)
    return rc if rc >= 0 else 128 - rc  # a rank killed by signal s: 128 + s, as a shell reports it


def main():
    a = parse()
    if a.launch_dry_run and os.environ.get("WORLD_SIZE"):
        # a launched rank of --launch-dry-run: report the rank environment, no GPU
        # (one write per line: the ranks share the parent's stdout)
        sys.stdout.write(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                                     "MASTER_PORT", "RT_BENCH_LAUNCHED")}) + "\n")
        sys.stdout.flush()
        # (tests: RT_BENCH_DRY_FAIL=r:code makes rank r exit with that code)
        fail = os.environ.get("RT_BENCH_DRY_FAIL", "")
        if fail and fail.split(":")[0] == os.environ.get("RANK"):
            return int(fail.split(":")[1])
        return 0
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ and not a.cpu_only:
        return launch_ranks(a)
    if os.environ.get("RT_BENCH_WATCHDOG"):
        # diagnostics: dump every thread's Python stack and exit if the run
        # takes longer than this many seconds
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["RT_BENCH_WATCHDOG"]), exit=True)
    if a.cpu_only:
        return cpu_only(a)
    import torch
    import torch.distributed as dist
    from cpp_cuda_raytracer_dev_amd import raytracer as R
    from cpp_cuda_raytracer_dev_amd.distributed import FrameGather, NativeFrameGather

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            print(f"bench.py: --gpus {a.gpus} needs torch.distributed.run with {a.gpus} processes", file=sys.stderr)
            return 2
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    multi = world > 1 or a.rehearse_gather
    if multi:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29531")
            dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
        else:
            dist.init_process_group("nccl", device_id=dev)
    w, h = a.width, a.height

    from cpp_cuda_raytracer_dev_amd import scenes
    pts, leafs, nodes, build_times = build_scene(a.scene)
    # the same tree built on this GPU (rt_kd_build_gpu):
    # first call (allocations included) and a warm one, byte-checked
    gb = []
    for _ in range(2):
        t0 = time.perf_counter()
        gnodes = R.kd_build_gpu(leafs, device=local)
        gb.append(time.perf_counter() - t0)
    build_times["kd_build_gpu_s"] = round(gb[1], 4)
    build_times["kd_build_gpu_s_first"] = round(gb[0], 4)
    build_times["kd_build_gpu_equals_host"] = gnodes.tobytes() == nodes.tobytes()
    del gnodes
    trixel = R.Trixel(len(pts), pts, device=local)
    trixel.set_kd_nodes(nodes)
    if a.treelet > 0:
        trixel.set_option(_lib_mod().RT_SCENE_TREELET_HEIGHT, a.treelet)
    if a.order >= 0:
        trixel.set_option(_lib_mod().RT_SCENE_ORDER, a.order)
    cam_kw = scenes.view(a.scene, a.view)
    cam = R.Camera(w, h, R.film_w(w, h), np.float32(.024), np.float32(.055), *cam_kw["pos"], *cam_kw["look_at"],
                   0.0, 1.0, 0.0, device=local)
    from cpp_cuda_raytracer_dev_amd import _lib
    # the counting frame runs the reference's DFS order (kernel 2); shadow
    # walks exist in kernel 3 only, whose accept count is the candidate count
    cam.set_option(_lib.RT_OPT_KERNEL, 3 if a.shadow else 2)
    cam.set_option(_lib.RT_OPT_TILE_ORDER, a.tile_order)
    obj = R.Object(trixel)
    cam.add_object(obj)
    xf = obj.quat.xform()
    stream = torch.cuda.Stream(device=dev)
    sptr = stream.cuda_stream
    tile = (world, rank)

    # Algorithmic counts of this rank's tiles (one untimed counting frame).
    npk = R.packed_pixels(w, h, world) if multi else w * h
    scratch = torch.zeros(npk, dtype=torch.int32, device=dev)
    sflag = R.RT_FLAG_SHADOW if a.shadow else 0
    masks = key_masks(a.animate) if a.animate else []
    if masks:
        # every timed frame has its own pose: count each of them (untimed),
        # replaying the same ticks on a separate motion state
        mo = R.ObjectMotion(cam.pos, cam.o_prop["n"], cam.o_prop["u"], cam.cam_speed)
        acc = np.zeros(5, np.float64)
        for i in range(a.warmup + a.steps):
            mo.tick(masks[i % len(masks)])
            if i >= a.warmup:
                cam.render_into(scratch, xform=mo.xform(), mode=a.mode, flags=R.RT_FLAG_COUNT | sflag,
                                tile=tile if multi else None, stream=sptr)
                torch.cuda.synchronize(dev)
                acc += cam.counters(reset=True)
        mo.close()
        cnt = acc / a.steps  # mean per frame
        # the same poses for the native loop (rt_frame_loop.xforms): pose i
        # is the object after tick i, frame i renders it
        mo = R.ObjectMotion(cam.pos, cam.o_prop["n"], cam.o_prop["u"], cam.cam_speed)
        poses = []
        for i in range(a.warmup + a.steps):
            mo.tick(masks[i % len(masks)])
            poses.append(np.asarray(mo.xform(), np.float32).reshape(12))
        mo.close()
        anim_xfs = np.stack(poses)
    else:
        cam.render_into(scratch, mode=a.mode, flags=R.RT_FLAG_COUNT | sflag, tile=tile if multi else None,
                        stream=sptr)
        torch.cuda.synchronize(dev)
        cnt = cam.counters(reset=True)
    root_passes = None
    if a.mode == 0 and not masks:
        # pixels whose root test passes (kernel 3's counting render with
        # debug bit 32 stops after the root test: counter [4]); the others'
        # root visits read no memory (the root box is a kernel argument), so
        # the roofline also reports the algorithmic bytes without them
        cam.set_option(_lib.RT_OPT_KERNEL, 3)
        cam.set_option(_lib.RT_OPT_DEBUG, 32)
        cam.render_into(scratch, mode=a.mode, flags=R.RT_FLAG_COUNT, tile=tile if multi else None, stream=sptr)
        torch.cuda.synchronize(dev)
        root_passes = int(cam.counters(reset=True)[4])
        cam.set_option(_lib.RT_OPT_DEBUG, 0)
    cam.set_option(_lib.RT_OPT_KERNEL, a.kernel)
    cam.set_option(_lib.RT_OPT_RAYS, a.rays)
    cam.set_option(_lib.RT_OPT_ITEMS, a.items)
    cam.set_option(_lib.RT_OPT_COARSE, a.coarse)
    cam.set_option(_lib.RT_OPT_SHADOW_ORDER, a.shadow_order)
    if a.flat >= 0:
        cam.set_option(_lib.RT_OPT_FLAT, a.flat)
    dbg_bits = (8 if a.side_coarse else 0) | a.debug_bits
    if dbg_bits:
        cam.set_option(_lib.RT_OPT_DEBUG, dbg_bits)
    cam.render_into(scratch, mode=a.mode, flags=sflag, tile=tile if multi else None,
                    stream=sptr)  # re-prepares layout
    torch.cuda.synchronize(dev)
    my_pix = int(np.count_nonzero(np.repeat(np.arange((h + 7) // 8) % world == rank, 8)[:h])) * w
    bytes_per_launch = B_INT * int(cnt[0]) + B_LEAF * int(cnt[1]) + B_HIT * int(cnt[2]) + B_PIX * my_pix

    loop_kind = a.loop
    # --inflight -1: multi-frame launches (RT_LOOP_MULTIFRAME: one grid holds
    # many frames' blocks, frame-major; N = 1, static scene, KD mode, no
    # shadow rays).  0 (auto, the default) takes them wherever they apply.
    # Against two lanes on one box (r04i, r04m, r04n): dragon 960x540 48.7k
    # -> 50.5k FPS over 1,000 frames (r04i, both without the settle); at
    # 1920x1080 the driver's 20 frames 10.11-10.20k -> 10.23-10.30k (knot),
    # 15.71k -> 15.96k (dragon), while over 1,000 frames two lanes stay 1-3 %
    # ahead (knot 10.60k vs 10.43-10.49k, dragon 16.90k vs 16.38k): the
    # second lane's first frame often cannot start before the first lane's
    # first frame ends (kernel traces), which a short window pays for
    can_mf = loop_kind == "native" and not multi and not a.animate and a.mode == 0 and not a.shadow
    multiframe = can_mf and a.inflight in (-1, 0)
    persistent = multiframe
    inflight = (2 if multiframe or a.inflight <= 0 else a.inflight) if loop_kind == "native" else 1
    if a.event_every <= 0:
        a.event_every = 8 if (multi or inflight > 1) else 1
    collective = a.collective
    gather_note = None

    def make_gather(kind):
        """(NativeFrameGather or None, FrameGather or None, render target)."""
        if multi and kind == "rccl":
            # two sets per frame in flight: a set's next render then waits
            # on a gather that finished long before (cross-queue waits that
            # are still pending cost ~10-15 us each)
            # (a multiple of the frames in flight: a set is always rendered
            # by the same lane, rt_run_frames requires it)
            nb = -(-max(a.pipeline, 2 * inflight) // inflight) * inflight
            g = NativeFrameGather(dist, w, h, dev, nbuf=max(inflight, min(nb, 8 // inflight * inflight)))
            # every rank must derive the same rectangle and options, or the
            # receive sizes would not match the sends
            g.verify(cam, xf, a.mode)
            return g, None, g.local[0]
        if multi:
            def unpack(g, f):
                R.unpack_bands(local, w, h, world, g, f, stream=torch.cuda.current_stream(dev).cuda_stream)
            f = FrameGather(dist, w, h, dev, kind, unpack=unpack)
            return None, f, f.local
        return None, None, [torch.zeros(w * h, dtype=torch.int32, device=dev) for _ in range(inflight)]

    try:
        ng, fg, out = make_gather(collective)
        failed = None
    except Exception as e:  # the library's communicator could not be set up on this rank
        ng, failed = None, e
    if multi and collective == "rccl":
        # every rank must take the same path: fall back to torch.distributed
        # gather everywhere when any rank failed
        bad = torch.tensor([1 if failed is not None else 0], dtype=torch.int64, device=dev)
        dist.all_reduce(bad)
        if int(bad[0]):
            if ng is not None:
                ng.close()
            gather_note = (f"native RCCL communicator failed on {int(bad[0])} rank(s)"
                           + (f" ({type(failed).__name__}: {failed})" if failed is not None else "")
                           + "; fell back to torch gather")
            collective = "gather"
            ng, fg, out = make_gather(collective)
    elif failed is not None:
        raise failed
    outs = out if isinstance(out, list) else [out]  # N=1: one target per frame in flight
    out = outs[0]
    cstream = torch.cuda.Stream(device=dev) if ng is not None else None

    def gathered_frame_ok(loop):
        """Rank 0's last gathered frame against a full frame rendered here (untimed),
        the verdict shared with every rank."""
        ok = torch.ones(1, dtype=torch.int64, device=dev)
        if rank == 0:
            got = ng.frames[loop.last_set()] if ng is not None else fg.frame
            full = torch.zeros(w * h, dtype=torch.int32, device=dev)
            cam.render_into(full, xform=xf, mode=a.mode, flags=sflag, stream=sptr)
            torch.cuda.synchronize(dev)
            ok[0] = int(torch.equal(got, full))
        dist.broadcast(ok, src=0)
        return bool(ok[0])

    class PyLoop:
        """The frame loop in Python (torch collectives, --animate, --loop python)."""

        def __init__(self):
            self.seq = 0
            self.tick = 0
            self.nbuf = len(ng.local) if ng is not None else 1
            if ng is not None:
                self.rendered = [torch.cuda.Event() for _ in range(self.nbuf)]
                self.sent = [torch.cuda.Event() for _ in range(self.nbuf)]
                for k in range(self.nbuf):
                    self.sent[k].record(cstream)

        def last_set(self):
            return (self.seq - 1) % self.nbuf

        def frame(self, timed):
            nonlocal xf
            if masks:  # one input tick, then the frame at the new pose
                obj.key_tick(masks[self.tick % len(masks)])
                self.tick += 1
                xf = obj.quat.xform()
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if timed else None
            if ng is not None:
                # frame j renders into buffer set j % nbuf once the gather that
                # last read it is done, then is gathered on the comm stream
                # while frame j + 1 renders
                k = self.seq % self.nbuf
                self.seq += 1
                stream.wait_event(self.sent[k])
                if ev:
                    ev[0].record(stream)
                cam.render_into(ng.local[k], xform=xf, mode=a.mode, flags=sflag, tile=tile, stream=sptr)
                if ev:
                    ev[1].record(stream)
                self.rendered[k].record(stream)
                cstream.wait_event(self.rendered[k])
                ng.gather(k, cam, xf, a.mode, cstream.cuda_stream)
                self.sent[k].record(cstream)
                return ev
            self.seq += 1
            with torch.cuda.stream(stream):
                if ev:
                    ev[0].record(stream)
                cam.render_into(out, xform=xf, mode=a.mode, flags=sflag, tile=tile if multi else None, stream=sptr)
                if ev:
                    ev[1].record(stream)
                if fg is not None:
                    fg.gather()
            return ev

        def run(self, n, time_frames):
            evs = []
            h0 = time.perf_counter()
            for i in range(n):
                e = self.frame(time_frames and i % a.event_every == 0)
                if e:
                    evs.append(e)
            host_ms = 1e3 * (time.perf_counter() - h0)
            torch.cuda.synchronize(dev)
            ms = [s0.elapsed_time(s1) for s0, s1 in evs]
            return (float(np.mean(ms)) if ms else 0.0), len(ms), host_ms

    def make_loop():
        if loop_kind == "native" and (not multi or ng is not None):
            return R.FrameLoop(cam, ng.local if ng is not None else outs, xform=xf, mode=a.mode, flags=sflag,
                               tile=tile if multi else None, render_stream=sptr, comm=ng,
                               comm_stream=cstream.cuda_stream if ng is not None else None,
                               event_every=a.event_every, inflight=-1 if persistent else inflight,
                               xforms=anim_xfs if masks else None)
        return PyLoop()

    loop = make_loop()
    loop.run(a.warmup, False) if isinstance(loop, PyLoop) else loop.run(a.warmup)
    torch.cuda.synchronize(dev)
    if multi and ng is not None and not gathered_frame_ok(loop):
        # the library's RCCL path has not been seen to work at N > 1 before
        # (ADVICE r01): on a wrong warm-up frame every rank falls back to
        # torch.distributed.gather and the line says so
        gather_note = "rccl warm-up frame differed from the single-GPU frame; fell back to torch gather"
        ng.close()
        collective = "gather"
        ng, fg, out = make_gather(collective)
        cstream = None
        loop = PyLoop()
        loop.run(a.warmup, False)
        torch.cuda.synchronize(dev)
    solo, batch_ms = None, []

    def measure_solo():
        """(median batch mean ms, frames per batch) of solo frames, or None."""
        if isinstance(loop, PyLoop) or inflight <= 1 or a.solo_frames <= 0:
            return None
        # the roofline's kernel time: solo frames (one in flight) back to
        # back, untimed, one event pair around the batch (per-frame event
        # pairs add ~5 us of queue time to each bracketed launch); the timed
        # frames overlap and share the GPU
        # (a moving object: the timed frames' own poses, all of them)
        nsolo = a.steps if masks else a.solo_frames
        sl = R.FrameLoop(cam, [ng.local[0] if ng is not None else outs[0]], xform=xf, mode=a.mode, flags=sflag,
                         tile=tile if multi else None, render_stream=sptr, event_every=0, inflight=1,
                         xforms=anim_xfs[a.warmup:] if masks else None)
        sl.run(20)
        # five batches (one for a moving object, whose batch is the timed
        # poses): the median batch mean is the kernel time, all are reported
        # (one batch of C3's 35 us frames is 7 ms, and batch means spread by
        # 10-30 % from run to run on one box)
        nbatch = 1 if masks else 5
        batch_ms.clear()
        for _ in range(nbatch):
            sl.seq.value = 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            sl.run(nsolo)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            batch_ms.append(e0.elapsed_time(e1) / nsolo)
        return float(np.median(batch_ms)), nsolo

    if a.solo_when == "before":
        solo = measure_solo()
    # Settle frames: the timed loop itself, untimed, for about --settle-ms of
    # GPU time right before the timed region.  Two frames in flight reach their
    # steady period only after ~20-35 ms of that load: knot 1080p pairs of
    # frames take 214 us at first and 186 us from ~35 ms on, while solo
    # frames stay at 105 us throughout (kernel traces r04e / r04k), so a
    # 20-frame window timed straight after the solo pass ran at 9.0-9.2k
    # FPS against 10.5k over 1000 frames (r04j, r04k).
    def run_untimed(n):
        loop.run(n, False) if isinstance(loop, PyLoop) else loop.run(n)

    settle = 0
    if a.settle_ms > 0 and masks and not isinstance(loop, PyLoop):
        # a moving object (native loop, whose frame k renders pose k): one
        # pass over the timed poses themselves, then the timed frames start
        # again at pose W (so a profile of the run averages the same poses)
        run_untimed(a.steps)
        torch.cuda.synchronize(dev)
        loop.seq.value = a.warmup
        settle = a.steps
    elif a.settle_ms > 0 and not masks:
        ts = time.perf_counter()
        run_untimed(50)
        torch.cuda.synchronize(dev)
        per = (time.perf_counter() - ts) / 50
        n = int(math.ceil(a.settle_ms * 1e-3 / max(per, 1e-6)))
        if multi:  # every rank renders (and gathers) the same frames
            tn = torch.tensor([n], dtype=torch.int64, device=dev)
            dist.all_reduce(tn, op=dist.ReduceOp.MAX)
            n = int(tn[0])
        run_untimed(n)
        settle = 50 + n
    # the GPU's idle time between the last untimed frame and the timed
    # region's start (diagnostic: clocks may fall in a long idle gap)
    g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)  # (the lanes' frames are not on `stream`)
    g0.record(stream)
    if multi:
        dist.barrier()
    torch.cuda.synchronize(dev)
    g1.record(stream)
    t0 = time.perf_counter()
    if isinstance(loop, PyLoop):
        kern_ms, n_ev, host_ms = loop.run(a.steps, True)
    else:
        kern_ms, n_ev, host_ms = loop.run(a.steps)
    torch.cuda.synchronize(dev)
    if multi:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    pre_timed_idle_us = 1e3 * g0.elapsed_time(g1)
    if a.solo_when == "after":
        solo = measure_solo()
    host_us_per_frame = 1e3 * host_ms / max(1, a.steps)
    if masks and not isinstance(loop, PyLoop):
        xf = anim_xfs[-1]  # the last timed frame's pose
    kern_ms_timed, n_ev_timed = kern_ms, n_ev
    if solo is not None and not persistent:
        kern_ms, n_ev = solo
    if persistent:
        # multi-frame launches do not overlap (one stream): the kernel time
        # is the timed launches' own, measured live -- every launch between
        # a pair of HIP events, their sum over the frames they rendered
        kern_label = (f"the timed region's multi-frame launches (RT_LOOP_MULTIFRAME), each between a pair of HIP events "
                      f"on the render stream: their total duration / the {n_ev} frames they rendered (kernel time per "
                      f"frame); kernel_ms_solo is one frame alone")
    elif solo is not None:
        kern_label = (f"median over {len(batch_ms)} batches of the mean period of {n_ev} solo frames back to back "
                      f"{a.solo_when} the timed region (one in flight; kernel + the launch gap, an upper bound of the "
                      f"kernel time); the timed frames keep {inflight} in flight")
    else:
        kern_label = f"{n_ev} of {a.steps} timed frames (every {max(1, a.event_every)})"
    kern_extra = ({"kernel_ms_solo": round(solo[0], 5),
                   "kernel_ms_solo_batches": [round(b, 5) for b in batch_ms],
                   "kernel_ms_avg_timed": round(kern_ms_timed, 5),
                   "kernel_ms_timed_frames": (f"{n_ev_timed} timed frames in multi-frame launches" if persistent else
                                              f"{n_ev_timed} of {a.steps} timed frames (every {a.event_every}), "
                                              f"each sharing the GPU with the other frames in flight")}
                  if solo is not None else {})
    # the device error word of this rank's timed frames (stack / pool
    # overflow, a far-group proof that failed): reported, and fatal below
    dev_err = cam.device_error(reset=True)
    # the timed frames' launch shape (before the per-frame loop below renders with its own)
    rays_used, fast_used = cam.get_option(_lib.RT_OPT_RAYS_USED), cam.get_option(_lib.RT_OPT_FAST_USED)
    frame_check = None
    if not multi and rank == 0:
        last = outs[loop.last_set()] if not isinstance(loop, PyLoop) else out
        frame_check = frame_check_n1(last.cpu().numpy().view(np.uint32), pts, nodes, cam_kw, a,
                                     xform=xf if masks else None)
    per_frame_loop = None
    if persistent and a.second_frames > 0:
        # VERDICT r04 item 7 / ADVICE r04: the headline batches copies of one
        # static frame per launch; the per-frame loop a moving scene would run
        # (rt_run_frames with two frames in flight on the render lanes, no
        # multi-frame launches) is timed here over its own frames, after the
        # same kind of settle, and reported beside it with its own frame check
        pl = R.FrameLoop(cam, outs, xform=xf, mode=a.mode, flags=sflag, render_stream=sptr, event_every=0,
                         inflight=inflight)
        ts = time.perf_counter()
        pl.run(50)
        torch.cuda.synchronize(dev)
        per = (time.perf_counter() - ts) / 50
        n2 = int(math.ceil(a.settle_ms * 1e-3 / max(per, 1e-6)))
        pl.run(n2)
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        _, _, host2 = pl.run(a.second_frames)
        torch.cuda.synchronize(dev)
        el2 = time.perf_counter() - t2
        err2 = cam.device_error(reset=True)
        check2 = frame_check_n1(outs[pl.last_set()].cpu().numpy().view(np.uint32), pts, nodes, cam_kw, a)
        per_frame_loop = {"loop": f"per-frame loop (rt_run_frames), {inflight} frames in flight on the library's "
                                  f"render lanes, no multi-frame launches",
                          "rays_per_wave": cam.get_option(_lib.RT_OPT_RAYS_USED),
                          "value": round(a.second_frames / el2, 2), "unit": "frames/s",
                          "mray_per_s": round(a.second_frames * w * h / el2 / 1e6, 2),
                          "frames": a.second_frames, "ms_per_frame": round(1e3 * el2 / a.second_frames, 5),
                          "settle_frames": 50 + n2, "host_us_per_frame": round(1e3 * host2 / a.second_frames, 2),
                          "device_err": err2, "frame_check": check2}
        if err2:
            dev_err = dev_err or err2
    ranks_info = None
    if multi:
        ok = gathered_frame_ok(loop)
        if rank == 0:
            frame_check = {"gathered_equals_single_gpu_frame": ok,
                           "collective": collective + (f", {len(ng.local)} buffer sets" if ng is not None else ""),
                           **({"note": gather_note} if gather_note else {})}
        # per rank: the rank count the communicator
        # reports, this rank's kernel time, and its gather alone -- 50
        # gathers of its last rendered buffer set back to back on the comm
        # stream, untimed, between one pair of HIP events (every rank takes
        # part in each: rank 0 receives, the peers pack and send)
        gather_us, comm_ranks = None, None
        if ng is not None:
            comm_ranks = ng.info()[0]
            k = loop.last_set()
            torch.cuda.synchronize(dev)
            dist.barrier()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cstream)
            for _ in range(50):
                ng.gather(k, cam, xf, a.mode, cstream.cuda_stream)
            e1.record(cstream)
            torch.cuda.synchronize(dev)
            gather_us = 1e3 * e0.elapsed_time(e1) / 50
        mine = {"rank": rank, "comm_ranks": comm_ranks, "kernel_us": round(1e3 * kern_ms, 2),
                "gather_us": round(gather_us, 2) if gather_us is not None else None,
                "host_us_per_frame": round(host_us_per_frame, 2)}
        ranks_info = [None] * world
        dist.all_gather_object(ranks_info, mine)
    full_walk = None
    if a.shadow and not masks:
        # shadow walks stop at their first occluder; the counting frame above
        # walked them in full (the oracle's counters).  Count the timed walk
        # (same push order) for the algorithmic bytes, untimed.
        full_walk = cnt
        cam.set_option(_lib.RT_OPT_DEBUG, 16 | dbg_bits)
        cam.render_into(scratch, xform=xf, mode=a.mode, flags=R.RT_FLAG_COUNT | sflag,
                        tile=tile if multi else None, stream=sptr)
        torch.cuda.synchronize(dev)
        cnt = cam.counters(reset=True)
        bytes_per_launch = B_INT * int(cnt[0]) + B_LEAF * int(cnt[1]) + B_HIT * int(cnt[2]) + B_PIX * my_pix
    errs = [dev_err]
    if multi:
        te = torch.zeros(world, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(te, torch.tensor([dev_err], dtype=torch.int64, device=dev))
        errs = [int(x) for x in te.cpu()]
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms_max = float(t[0]), float(t[1])
        tb = torch.tensor([bytes_per_launch], dtype=torch.float64, device=dev)
        dist.all_reduce(tb, op=dist.ReduceOp.MAX)
        th = torch.tensor([int(cnt[3])], dtype=torch.float64, device=dev)
        dist.all_reduce(th, op=dist.ReduceOp.SUM)
        hits_all = int(th[0])
    else:
        kern_ms_max = kern_ms
        hits_all = int(cnt[3])
    # rays per frame: every pixel's primary ray, plus a shadow ray per hit
    rays_per_frame = w * h + (hits_all if a.shadow else 0)

    solo_before = (20 + len(batch_ms) * solo[1]) if (solo is not None and a.solo_when == "before") else 0
    if persistent:
        loop_label = ("multi-frame launches (RT_LOOP_MULTIFRAME): up to 128 copies of the same static frame per "
                      "k_trace_kd3 launch, frame-major; a batching mode for a static scene, not a per-frame loop")
    elif isinstance(loop, PyLoop):
        loop_label = "per-frame loop from Python, one frame at a time" + (" + gather" if multi else "")
    else:
        loop_label = (f"per-frame loop (rt_run_frames), {inflight} frame(s) in flight on the library's render lanes"
                      + (" + RCCL gather to rank 0 on the comm lane" if ng is not None else
                         " + torch gather" if multi else ""))
    rc = 0
    if rank == 0:
        fps = a.steps / elapsed
        achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
        tests = w * h * len(pts)  # flat list: every ray against every triangle
        tflops = FLOPS_PER_TEST * tests / (kern_ms * 1e-3) / 1e12
        # counter-based figures of this configuration from the committed PMC
        # passes (tools/pmc_plan.py: one frame in flight, or with --own the
        # multi-frame launches of this loop, key suffix _mf; the same kernel),
        # stamped with the build id of the library they measured
        traffic, valu_util, pmc_key, pmc_build, vmem_util, vmem = None, None, None, None, None, None
        if os.path.exists(a.traffic_json):
            try:
                tj = json.load(open(a.traffic_json))
                key = (f"{a.scene}_{w}x{h}_m{a.mode}_n{world}" + ("_shadow" if a.shadow else "")
                       + ("" if a.view == "default" else f"_{a.view}") + (f"_anim{a.steps}" if a.animate else "")
                       + ("_mf" if persistent else ""))  # multi-frame launches: passes of that loop
                ent = tj.get(key) or {}
                # HBM bytes per frame (older entries: per launch of one frame)
                traffic = ent.get("hbm_bytes_per_frame", ent.get("hbm_bytes_per_launch"))
                pmc_fpd = ent.get("frames_per_dispatch", 1.0)
                valu_util = ent.get("valu_issue_util")
                vmem_util, vmem = ent.get("vmem_util"), ent.get("vmem")
                pmc_build = ent.get("build_id")
                pmc_key = key if ent else None
            except Exception:
                traffic = valu_util = pmc_key = pmc_build = vmem_util = vmem = None
                pmc_fpd = None
        kern_s = kern_ms * 1e-3
        # compulsory bytes of one frame: every record of the scene read once
        # (n - 1 interior records and n triangle records, 64 B each) and the
        # frame written once (verdict r05 item 4)
        compulsory = 64 * (2 * len(pts) - 1) + 4 * my_pix
        stale = pmc_key is not None and pmc_build != _lib.build_id()
        hbm_util = traffic / kern_s / (HBM_PEAK_GBS * 1e9) if traffic else None
        # roofline.frac is the utilisation of the binding resource (VERDICT
        # r03 item 1): the counter HBM bytes over this run's kernel time
        # against 8 TB/s, or the VALU issue share of the chip's SIMD cycles,
        # whichever is higher; the SURVEY.md 8d algorithmic (demand) figure
        # moves to demand_frac (L1/L2 serve most of those bytes, so it can
        # exceed 1)
        # Round 6 (verdict r05 item 4): the vector memory path is the third
        # candidate -- the texture data unit's busy share of CU cycles
        # (TD_TD_BUSY; the address unit's TA_TA_BUSY beside it), which binds
        # the 1080p walks (tools/ubench_l1.hip: a wave's 16-B loads cost the
        # unit max(1, distinct 128-B lines) cycles per 4-lane quad)
        phys = [(u, b) for u, b in ((hbm_util, "hbm"), (valu_util, "valu"), (vmem_util, "vmem")) if u is not None]
        binding = max(phys) if phys else (None, None)
        util = {
            "hbm_util": round(hbm_util, 4) if hbm_util is not None else None,
            "valu_issue_util": valu_util,
            "vmem_util": vmem_util,
            **({"vmem_per_cu_cycle": vmem} if vmem else {}),
            "util_source": (("STALE (measured on build " + str(pmc_build)[:16] + ", not this library): " if stale else "")
                            + f"profiles/pmc_traffic.json[{pmc_key}]: HBM bytes per frame (FETCH_SIZE x2 + WRITE_SIZE, "
                            "MI355X_MICROARCH.md) / this run's kernel time per frame / 8 TB/s; SQ_INSTS_VALU x 2 "
                            "cycles / (1,024 SIMDs x GRBM_GUI_ACTIVE / 8), over the passes' launches of this loop "
                            f"({pmc_fpd} frames per launch)") if pmc_key else
                           "no committed PMC passes for this configuration",
            "util_build_id": pmc_build,
            "util_stale": stale if pmc_key else None,
        }
        res = {
            "metric": METRIC,
            #  the metric string is BASELINE.json's; since round 3
            # the default workload is the knot stand-in, named in
            # config.workload (the displaced-sphere blob is --scene dragon)
            "metric_workload": (f"{a.scene}{' stand-in' if a.scene in scenes.STANDINS else ''} {w}x{h}"
                                + ("" if a.view == "default" else f" {a.view} view")),
            "value": round(fps, 2),
            "unit": "frames/s",
            "mray_per_s": round(fps * rays_per_frame / 1e6, 2),
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            # every untimed frame of the timed loop and the solo pass that ran
            # before the timed region
            "warmup_effective": a.warmup + settle + solo_before,
            "warmup_breakdown": {"warmup": a.warmup, "settle": settle, "solo_pass": solo_before},
            "loop": loop_label,
            "ms_per_step": round(1e3 * elapsed / a.steps, 5),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": data_label(a.scene),
            "config": {
                "workload": f"{a.scene}{' stand-in' if a.scene in scenes.STANDINS else ''} {w}x{h}"
                            + ("" if a.view == "default" else f" ({a.view} view)")
                            + f", {'KD traversal' if a.mode == 0 else 'flat list'}, "
                            + ("primary + one shadow ray per hit" if a.shadow else "primary rays")
                            + " + Phong, u32 frame on GPU 0"
                            + (f", object moved by keys {a.animate!r} (one tick per frame)" if masks else ""),
                "rays_per_frame": rays_per_frame,
                "scene": (f"synthetic {a.scene} stand-in, {len(pts)} triangles (seed 20221015)"
                          if a.scene in scenes.STANDINS else f"{a.scene}.ply (the reference's mesh), {len(pts)} triangles"),
                "resolution": [w, h],
                "view": {"name": a.view, **cam_kw},
                "coverage": round(hits_all / (w * h), 5),
                "parallelism": f"screen bands x{world}" + ((" + RCCL send/recv to rank 0, pipelined" if collective == "rccl"
                                                         else f" + torch {collective} to rank 0") if multi else ""),
            },
            "roofline": ({
                "bound": "valu",
                "achieved": round(tflops, 2),
                "peak": VALU_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(tflops / VALU_PEAK_TFLOPS, 4),
                "traffic": None,
                **util,
                "kernel": "k_trace_flat",
                "kernel_form": cam.get_option(_lib.RT_OPT_FLAT),
                "kernel_ms_avg": round(kern_ms, 5),
                "kernel_ms_frames": kern_label,
                "kernel_ms_avg_max_rank": round(kern_ms_max, 5),
                **kern_extra,
                "tests_per_launch": tests,
                "flops_per_launch": FLOPS_PER_TEST * tests,
                "divides_per_launch": tests,
                "peak_unpacked": VALU_PEAK_UNPACKED_TFLOPS,
                "flops_model": "28 FP32 flops + 1 divide per ray-triangle test x npix x ntri (SURVEY.md 8d, "
                               "TD/Trixel.cu:173-209); peak = non-FMA FP32 issue with packed v_pk_* "
                               "(157.3 TF FMA spec / 2), 39.3 unpacked",
                "counts_per_launch": {"leaf_tests": int(cnt[1]), "accept": int(cnt[2]), "hit_pixels": int(cnt[3]),
                                      "pixels": my_pix},
            } if a.mode == 1 else {
                # the binding resource (see util above); with no committed
                # counters for this configuration frac is null
                "bound": binding[1] or "hbm",
                "achieved": (round(traffic / kern_s / 1e9, 1) if binding[1] == "hbm" else
                             round(valu_util * VALU_PEAK_TFLOPS, 2) if binding[1] == "valu" else
                             round(vmem_util, 4) if binding[1] == "vmem" else None),
                "peak": (VALU_PEAK_TFLOPS if binding[1] == "valu" else 1.0 if binding[1] == "vmem" else HBM_PEAK_GBS),
                "unit": ("T VALU lane-ops/s" if binding[1] == "valu" else
                         "busy cycles of the CU's texture data unit per CU cycle" if binding[1] == "vmem" else "GB/s"),
                "frac": round(binding[0], 4) if binding[0] is not None else None,
                "frac_rule": "max(hbm_util, valu_issue_util, vmem_util): L2-miss (fabric) bytes per frame / kernel time "
                             "/ 8 TB/s; the VALU issue share (SQ_INSTS_VALU x 2 cycles over 1,024 SIMDs' cycles; a "
                             "VALU wave64 instruction is 64 lane-ops, 1,024 SIMDs x 2.4 GHz x 64 / 2 = 78.6 T/s); the "
                             "texture data unit's busy share of CU cycles (TD_TD_BUSY_sum / (GRBM_GUI_ACTIVE / 8 x 256))",
                "traffic": traffic,
                # the counter bytes are L2-miss (fabric) requests: MI355X_MICROARCH.md says FETCH_SIZE counts
                # Infinity-Cache hits too, and the scene (compulsory_bytes) fits the 256 MB cache, so most of
                # them never reach HBM (verdict r05 item 4)
                "traffic_kind": "L2-miss fabric bytes (FETCH_SIZE x2 + WRITE_SIZE per frame; Infinity-Cache hits included)",
                "compulsory_bytes": compulsory,
                "traffic_over_compulsory": round(traffic / compulsory, 3) if traffic else None,
                "compulsory_model": "64 B per interior record (n - 1) + 64 B per triangle record (n) + 4 B per pixel "
                                    "of the frame written",
                **util,
                "demand_achieved": round(achieved, 1),
                "demand_frac": round(achieved / HBM_PEAK_GBS, 4),
                "demand_unit": "GB/s of SURVEY.md 8d algorithmic bytes (every visited record counted per visit; "
                               "L1/L2 serve most of them, so this can exceed 1)",
                **({"demand_frac_excl_root_misses": round((bytes_per_launch - B_INT * (my_pix - root_passes)) / kern_s
                                                          / 1e9 / HBM_PEAK_GBS, 4),
                    "root_pass_pixels": root_passes} if root_passes is not None and not multi else {}),
                "kernel": {2: "k_trace_kd2", 3: "k_trace_kd3"}[a.kernel] if a.mode == 0
                          else "k_trace_flat",
                "kernel_options": {"kernel": a.kernel, "tile_order": a.tile_order,
                                   "rays_per_wave": rays_used,
                                   "fast_walks": fast_used,
                                   "rays_per_wave_option": a.rays,
                                   "record_order": trixel.get_option(_lib.RT_SCENE_ORDER),
                                   "treelet_height": trixel.get_option(_lib.RT_SCENE_TREELET_HEIGHT),
                                   "items_per_lane": a.items, "coarse_groups_per_wave": a.coarse,
                                   "shadow": a.shadow,
                                   **({"shadow_push_order": cam.get_option(_lib.RT_OPT_SHADOW_ORDER),
                                       "shadow_push_order_mode": "timed" if a.shadow_order < 0 else "fixed"}
                                      if a.shadow else {})},
                "kernel_ms_avg": round(kern_ms, 5),
                "kernel_ms_frames": kern_label,
                "kernel_ms_avg_max_rank": round(kern_ms_max, 5),
                **kern_extra,
                "algorithmic_bytes_per_launch": bytes_per_launch,
                # with frames in flight, launches overlap: the bytes of one
                # frame over the frame period (elapsed / steps) as well
                "demand_achieved_per_frame_period": round(bytes_per_launch / (elapsed / a.steps) / 1e9, 1),
                "demand_frac_per_frame_period": round(bytes_per_launch / (elapsed / a.steps) / 1e9 / HBM_PEAK_GBS, 4),
                "counts_per_launch": {"interior": int(cnt[0]), "leaf": int(cnt[1]), "accept": int(cnt[2]),
                                      "hit_pixels": int(cnt[3]), "pixels": my_pix},
                **({"counts_full_shadow_walk": {"interior": int(full_walk[0]), "leaf": int(full_walk[1]),
                                                "accept": int(full_walk[2])}} if full_walk is not None else {}),
                "bytes_model": "36*V_int + 40*V_leaf + 24*H + 4*P (SURVEY.md 8d)",
            }),
            "device_err": errs if multi else dev_err,
            **({"ranks": ranks_info} if ranks_info is not None else {}),
            "host": {"us_per_frame": round(host_us_per_frame, 2), "pre_timed_idle_us": round(pre_timed_idle_us, 1),
                     "settle_frames": settle,
                     "loop": "native (rt_run_frames)"
                     if not isinstance(loop, PyLoop) else "python",
                     "frames_in_flight": ("multi-frame launches" if persistent else inflight)
                     if not isinstance(loop, PyLoop) else 1,
                     "what": "host time spent enqueueing the timed frames / steps (rank 0)"},
            "kd_build": build_times,
            # build provenance: SHA-256 of the library's sources and flags
            # (rt_build_id; _lib refuses a library whose id is not this tree's)
            "build_id": _lib.build_id(),
        }
        if frame_check is not None:
            res["frame_check"] = frame_check
        if per_frame_loop is not None:
            res["per_frame_loop"] = per_frame_loop
            if per_frame_loop["frame_check"].get("matches_oracle") is False:
                frame_check = per_frame_loop["frame_check"]
        if a.deliver and world == 1:
            res["delivery"] = delivery(cam, R, torch, dev, w, h, xf, a.mode, sflag, a.steps, a.warmup)
        if not a.no_cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline(pts, nodes, w, h, a.cpu_seconds, cpu_threads(a.cpu_threads), a.mode,
                                              a.shadow, rays_per_frame, cam_kw, build_times)
        else:
            res["cpu_baseline"] = None
        print(json.dumps(res), flush=True)
        bad = [e for e in errs if e]
        fc = (frame_check or {}).get("matches_oracle", (frame_check or {}).get("gathered_equals_single_gpu_frame"))
        if bad:
            print(f"bench.py: device error word {errs} after the timed frames", file=sys.stderr)
            rc = 3
        elif fc is False:
            print("bench.py: frame_check failed", file=sys.stderr)
            rc = 4
    if multi:
        dist.barrier()
    # explicit teardown: every device object this run
    # made is released here, after a device-wide synchronisation, while the
    # HIP runtime and any profiler tool are fully alive -- not by finalisers
    # at interpreter exit (the raytracer finalisers are no-ops then)
    torch.cuda.synchronize(dev)
    release(ng, cam, obj, trixel)
    torch.cuda.synchronize(dev)
    if multi:
        dist.destroy_process_group()
    maps = os.environ.get("RT_BENCH_MAPS")
    if maps:  # diagnostics: this process's mappings, to symbolise a crash report's addresses
        with open(maps, "w") as fp, open("/proc/self/maps") as src:
            fp.write(src.read())
    return rc


def release(ng, cam, obj, trixel):
    """Closes the run's library handles in dependency order: the RCCL
    communicator, the camera (its streams, events, buffers), the object's
    motion state, then the scene."""
    for h in (ng, cam, getattr(obj, "motion", None), trixel):
        if h is not None:
            h.close()


if __name__ == "__main__":
    sys.exit(main())
