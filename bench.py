#!/usr/bin/env python3
"""Benchmark: frames/s and Mray/s at 1920x1080 on the dragon (stand-in),
KD traversal, 1..N MI355X GPUs (BASELINE.json metric; configs C3/C4).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

A step is one frame: bg fill -> primary rays -> KD traversal -> Moller-
Trumbore -> Phong into the u32 frame (one fused kernel), plus, for N > 1,
the RCCL gather to rank 0 of every rank's screen bands (the part of them
not provably background) and the frame assembly kernel there, pipelined
with the next frame's render.  Frames are fixed-size (1920x1080), so N > 1 is strong
scaling.  The scene is the seeded synthetic stand-in for
dragon_vrip_mod.ply (missing from the reference; 871,414 triangles).
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/sec + Mray/s at 1920×1080, Stanford dragon 800k tris, 1/2/4/8 GPU"
W, H = 1920, 1080
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# bytes per interior visit, leaf visit, accepted hit, pixel
B_INT, B_LEAF, B_HIT, B_PIX = 36, 40, 24, 4


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--scene", default="dragon", choices=["dragon", "happy"])
    ap.add_argument("--width", type=int, default=W)
    ap.add_argument("--height", type=int, default=H)
    ap.add_argument("--mode", type=int, default=0, help="0 KD, 1 flat list")
    ap.add_argument("--collective", default="rccl", choices=["rccl", "gather", "allgather"],
                    help="N>1 frame gather: rccl = the library's own RCCL send/recv + unpack (rt_comm_*, "
                         "pipelined); gather / allgather = torch.distributed collectives, one frame at a time")
    ap.add_argument("--rehearse-gather", action="store_true",
                    help="one process: run the N>1 frame loop (process group, gather, frame check) with one rank, "
                         "to rehearse the multi-GPU path on a one-GPU machine; not a bench line")
    ap.add_argument("--pipeline", type=int, default=2,
                    help="rccl: buffer sets in flight (frame i+1 renders while frame i is gathered)")
    ap.add_argument("--kernel", type=int, default=3,
                    help="KD kernel: 1 per-lane DFS (own-box records), 2 per-lane DFS (child-box records), "
                         "3 wave-cooperative item pool")
    ap.add_argument("--tile-order", type=int, default=3,
                    help="0 XCD-contiguous, 1 natural, 2 centre-out, 3 by the cost an earlier frame measured")
    ap.add_argument("--rays", type=int, default=16, help="kernel 3: pixels per wave (64, 32, 16, 8)")
    ap.add_argument("--items", type=int, default=2, help="kernel 3: items each lane pops per iteration (1, 2)")
    ap.add_argument("--coarse", type=int, default=8,
                    help="kernel 3: 8x8 groups per wave outside the root box's screen rectangle (0 = off)")
    ap.add_argument("--event-every", type=int, default=0,
                    help="bracket every Nth timed frame with HIP events for the kernel time (each pair costs "
                         "queue time, so N > 1 keeps the frame rate closer to the uninstrumented one); 0 = every frame "
                         "at one GPU, every 8th with more, where a frame is a few tens of microseconds")
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
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample length")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def build_scene(name):
    from cpp_cuda_raytracer_dev_amd import raytracer as R, scenes
    v, f = scenes.standin(name)
    pts, n, leafs = R.assemble_mesh(v, f)
    nodes = R.kd_build(leafs)
    return pts, leafs, nodes


def cpu_baseline(pts, nodes, w, h, seconds, threads, mode, shadow=False, rays_per_frame=None):
    """The oracle (C restatement, -O2, OpenMP over rows) on the same frame,
    repeated for ~`seconds`.  Test infrastructure: the checker, timed beside
    the GPU; never part of the product path."""
    from oracle import _oracle as O
    on = np.zeros(len(nodes), O.NODE_DTYPE)
    for k in nodes.dtype.names:
        on[k] = nodes[k]
    s = O.Scene(pts, O.default_rad(len(pts)), on if mode == 0 else None, O.camera(w, h))
    rows = (0, h)
    if mode == 1:  # flat list is O(npix*ntri): sample a band of rows
        rows = (h // 2 - 4, h // 2 + 4)
    frames, t0 = 0, time.perf_counter()
    while True:
        s.render(mode, rows=rows, nthreads=threads, want_hit=False, shadow=shadow)
        frames += 1
        if time.perf_counter() - t0 >= seconds and frames >= 2:
            break
    dt = time.perf_counter() - t0
    s.close()
    frac = (rows[1] - rows[0]) / h
    fps = frames * frac / dt
    return {"value": round(fps, 3), "unit": "frames/s", "cores": threads, "kind": "port",
            "mray_per_s": round(fps * (rays_per_frame or w * h) / 1e6, 3),
            "sample": f"{frames} x rows {rows[0]}-{rows[1]} of the same {w}x{h} frame, oracle/oracle.c "
                      f"(-O2 -ffp-contract=off, OpenMP {threads} threads), {dt:.1f} s"}


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


def main():
    a = parse()
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

    pts, leafs, nodes = build_scene(a.scene)
    trixel = R.Trixel(len(pts), pts, device=local)
    trixel.set_kd_nodes(nodes)
    cam = R.Camera.default(w, h, device=local)
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
    else:
        cam.render_into(scratch, mode=a.mode, flags=R.RT_FLAG_COUNT | sflag, tile=tile if multi else None,
                        stream=sptr)
        torch.cuda.synchronize(dev)
        cnt = cam.counters(reset=True)
    cam.set_option(_lib.RT_OPT_KERNEL, a.kernel)
    cam.set_option(_lib.RT_OPT_RAYS, a.rays)
    cam.set_option(_lib.RT_OPT_ITEMS, a.items)
    cam.set_option(_lib.RT_OPT_COARSE, a.coarse)
    cam.set_option(_lib.RT_OPT_SHADOW_ORDER, a.shadow_order)
    if a.side_coarse:
        cam.set_option(_lib.RT_OPT_DEBUG, 8)
    cam.render_into(scratch, mode=a.mode, flags=sflag, tile=tile if multi else None,
                    stream=sptr)  # re-prepares layout
    torch.cuda.synchronize(dev)
    my_pix = int(np.count_nonzero(np.repeat(np.arange((h + 7) // 8) % world == rank, 8)[:h])) * w
    bytes_per_launch = B_INT * int(cnt[0]) + B_LEAF * int(cnt[1]) + B_HIT * int(cnt[2]) + B_PIX * my_pix

    ng = None
    if multi and a.collective == "rccl":
        fg = None
        ng = NativeFrameGather(dist, w, h, dev, nbuf=max(1, a.pipeline))
        nbuf = len(ng.local)
        cstream = torch.cuda.Stream(device=dev)
        rendered = [torch.cuda.Event() for _ in range(nbuf)]
        sent = [torch.cuda.Event() for _ in range(nbuf)]
        for k in range(nbuf):
            sent[k].record(cstream)
        out = ng.local[0]
    elif multi:
        def unpack(g, f):
            R.unpack_bands(local, w, h, world, g, f, stream=torch.cuda.current_stream(dev).cuda_stream)
        fg = FrameGather(dist, w, h, dev, a.collective, unpack=unpack)
        out = fg.local
    else:
        fg = None
        out = torch.zeros(w * h, dtype=torch.int32, device=dev)

    if a.event_every <= 0:
        a.event_every = 8 if multi else 1
    timed_frames = list(range(0, a.steps, max(1, a.event_every)))
    ev = {i: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for i in timed_frames}

    tick = [0]
    seq = [0]

    def frame(i=None):
        nonlocal xf
        if masks:  # one input tick, then the frame at the new pose
            obj.key_tick(masks[tick[0] % len(masks)])
            tick[0] += 1
            xf = obj.quat.xform()
        if ng is not None:
            # frame j renders into buffer set j % nbuf once the gather that
            # last read it is done, then is gathered on the comm stream while
            # frame j + 1 renders
            k = seq[0] % nbuf
            seq[0] += 1
            stream.wait_event(sent[k])
            if i in ev:
                ev[i][0].record(stream)
            cam.render_into(ng.local[k], xform=xf, mode=a.mode, flags=sflag, tile=tile, stream=sptr)
            if i in ev:
                ev[i][1].record(stream)
            rendered[k].record(stream)
            cstream.wait_event(rendered[k])
            ng.gather(k, cam, xf, a.mode, cstream.cuda_stream)
            sent[k].record(cstream)
            return
        with torch.cuda.stream(stream):
            if i in ev:
                ev[i][0].record(stream)
            cam.render_into(out, xform=xf, mode=a.mode, flags=sflag, tile=tile if multi else None,
                            stream=sptr)
            if i in ev:
                ev[i][1].record(stream)
            if fg is not None:
                fg.gather()

    for _ in range(a.warmup):
        frame()
    torch.cuda.synchronize(dev)
    if multi:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        frame(i)
    torch.cuda.synchronize(dev)
    if multi:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    frame_check = None
    if multi and rank == 0:
        # the last gathered frame against a full frame rendered here (untimed)
        got = ng.frames[(seq[0] - 1) % nbuf] if ng is not None else fg.frame
        full = torch.zeros(w * h, dtype=torch.int32, device=dev)
        cam.render_into(full, xform=xf, mode=a.mode, flags=sflag, stream=sptr)
        torch.cuda.synchronize(dev)
        frame_check = bool(torch.equal(got, full))
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in ev.values()]))
    full_walk = None
    if a.shadow and not masks:
        # shadow walks stop at their first occluder; the counting frame above
        # walked them in full (the oracle's counters).  Count the timed walk
        # (same push order) for the algorithmic bytes, untimed.
        full_walk = cnt
        cam.set_option(_lib.RT_OPT_DEBUG, 16 | (8 if a.side_coarse else 0))
        cam.render_into(scratch, xform=xf, mode=a.mode, flags=R.RT_FLAG_COUNT | sflag,
                        tile=tile if multi else None, stream=sptr)
        torch.cuda.synchronize(dev)
        cnt = cam.counters(reset=True)
        bytes_per_launch = B_INT * int(cnt[0]) + B_LEAF * int(cnt[1]) + B_HIT * int(cnt[2]) + B_PIX * my_pix
    if multi:
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

    if rank == 0:
        fps = a.steps / elapsed
        achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
        traffic = None
        if os.path.exists(a.traffic_json):
            try:
                tj = json.load(open(a.traffic_json))
                key = f"{a.scene}_{w}x{h}_m{a.mode}_n{world}"
                traffic = tj.get(key, {}).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        res = {
            "metric": METRIC,
            "value": round(fps, 2),
            "unit": "frames/s",
            "mray_per_s": round(fps * rays_per_frame / 1e6, 2),
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1e3 * elapsed / a.steps, 5),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": f"{a.scene} stand-in {w}x{h}, {'KD traversal' if a.mode == 0 else 'flat list'}, "
                            + ("primary + one shadow ray per hit" if a.shadow else "primary rays")
                            + " + Phong, u32 frame on GPU 0"
                            + (f", object moved by keys {a.animate!r} (one tick per frame)" if masks else ""),
                "rays_per_frame": rays_per_frame,
                "scene": f"synthetic {a.scene} stand-in, {len(pts)} triangles (seed 20221015)",
                "resolution": [w, h],
                "parallelism": f"screen bands x{world}" + ((" + RCCL send/recv to rank 0, pipelined" if a.collective == "rccl"
                                                         else f" + torch {a.collective} to rank 0") if multi else ""),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": {1: "k_trace_kd", 2: "k_trace_kd2", 3: "k_trace_kd3"}[a.kernel] if a.mode == 0
                          else "k_trace_flat",
                "kernel_options": {"kernel": a.kernel, "tile_order": a.tile_order, "rays_per_wave": a.rays,
                                   "items_per_lane": a.items, "coarse_groups_per_wave": a.coarse,
                                   "shadow": a.shadow,
                                   **({"shadow_push_order": cam.get_option(_lib.RT_OPT_SHADOW_ORDER),
                                       "shadow_push_order_mode": "timed" if a.shadow_order < 0 else "fixed"}
                                      if a.shadow else {})},
                "kernel_ms_avg": round(kern_ms, 5),
                "kernel_ms_frames": f"{len(ev)} of {a.steps} timed frames (every {max(1, a.event_every)})",
                "kernel_ms_avg_max_rank": round(kern_ms_max, 5),
                "algorithmic_bytes_per_launch": bytes_per_launch,
                "counts_per_launch": {"interior": int(cnt[0]), "leaf": int(cnt[1]), "accept": int(cnt[2]),
                                      "hit_pixels": int(cnt[3]), "pixels": my_pix},
                **({"counts_full_shadow_walk": {"interior": int(full_walk[0]), "leaf": int(full_walk[1]),
                                                "accept": int(full_walk[2])}} if full_walk is not None else {}),
                "bytes_model": "36*V_int + 40*V_leaf + 24*H + 4*P (SURVEY.md 8d)",
            },
        }
        if frame_check is not None:
            res["frame_check"] = {"gathered_equals_single_gpu_frame": frame_check,
                                  "collective": a.collective + (f", {nbuf} buffer sets" if ng is not None else "")}
        if a.deliver and world == 1:
            res["delivery"] = delivery(cam, R, torch, dev, w, h, xf, a.mode, sflag, a.steps, a.warmup)
        if not a.no_cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline(pts, nodes, w, h, a.cpu_seconds, a.cpu_threads, a.mode, a.shadow,
                                              rays_per_frame)
        else:
            res["cpu_baseline"] = None
        print(json.dumps(res), flush=True)
    if multi:
        dist.barrier()
        if ng is not None:
            ng.close()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
