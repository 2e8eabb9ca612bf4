#!/usr/bin/env python3
"""Project the N-GPU frame on one GPU: render each rank's screen bands
(rt_tile{N, r}) alone, timed with HIP events over many frames, for N = 1, 2,
4, 8.  A rank's render time bounds its frame time at N GPUs (the gather
overlaps the next frame's render), so max over r is the per-frame floor of the
multi-GPU run and w*h / max the best N-GPU frame rate the render allows.  Also
reports the bytes each peer sends to rank 0 (the rectangle gather).

    python tools/project_ranks.py [--scene dragon] [--width 1920 --height 1080] [--frames 300] [--rays 0]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def wave_stamps(cam, _lib, R, torch, st, n, r, npk):
    """Per-wave (start, end, pool iterations, items popped) of one render of
    rank r's tile (debug bit 2; s_memrealtime, 100 MHz): the longest waves."""
    buf = torch.zeros(npk, dtype=torch.int32, device="cuda:0")
    cam.set_option(_lib.RT_OPT_DEBUG, 2)
    cam.render_into(buf, tile=(n, r), stream=st.cuda_stream)
    st.synchronize()
    raw = np.zeros(3 * 4 * 400000, np.uint64)
    got = _lib.lib().rt_camera_debug_read(cam._h, _lib.ptr(raw), len(raw))
    cam.set_option(_lib.RT_OPT_DEBUG, 0)
    rec = raw[:got].reshape(-1, 3).astype(np.int64)
    rec = rec[rec[:, 1] > 0]
    t0 = rec[:, 0].min()
    dur = (rec[:, 1] - rec[:, 0]) * 10e-3
    end = (rec[:, 1] - t0) * 10e-3
    it = rec[:, 2] & 0xFFFFFFFF
    fine = it != 0xFFFFFFFF
    top = np.argsort(-end)[:8]
    return {"waves": int(fine.sum()), "kernel_span_us": float(end.max()),
            "iters_p50_p99_max": [float(np.percentile(it[fine], q)) for q in (50, 99, 100)],
            "dur_us_p50_p99_max": [float(np.percentile(dur[fine], q)) for q in (50, 99, 100)],
            "us_per_iter_of_longest": [round(float(dur[i] / max(1, it[i])), 3) for i in np.argsort(-dur)[:8]],
            "latest_finishers": [{"start_us": round(float((rec[i, 0] - t0) * 10e-3), 2), "dur_us": round(float(dur[i]), 2),
                                  "iters": int(it[i]), "popped": int(rec[i, 2] >> 32)} for i in top]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="dragon")
    ap.add_argument("--view", default="default")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--rays", type=int, default=0)
    ap.add_argument("--items", type=int, default=2)
    ap.add_argument("--inflight", type=int, default=1,
                    help="frames in flight per rank (rt_frame_loop.inflight); the frame period then bounds the "
                         "rank, not the kernel time")
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--out", default="")
    ap.add_argument("--lib", default="", help="an experiment build of librt_mi355x.so (tools/build_variants.sh)")
    ap.add_argument("--stamps", action="store_true",
                    help="also record per-wave clocks of the slowest rank at each N (pool iterations, duration)")
    a = ap.parse_args()
    import torch
    from cpp_cuda_raytracer_dev_amd import _lib, raytracer as R, scenes
    if a.lib:
        _lib.LIB_PATH = os.path.abspath(a.lib)
    import bench
    pts, leafs, nodes, _ = bench.build_scene(a.scene)
    w, h = a.width, a.height
    t = R.Trixel(len(pts), pts)
    t.set_kd_nodes(nodes)
    kw = scenes.view(a.scene, a.view)
    cam = R.Camera(w, h, R.film_w(w, h), np.float32(.024), np.float32(.055), *kw["pos"], *kw["look_at"],
                   0.0, 1.0, 0.0)
    obj = R.Object(t)
    cam.add_object(obj)
    cam.set_option(_lib.RT_OPT_RAYS, a.rays)
    cam.set_option(_lib.RT_OPT_ITEMS, a.items)
    st = torch.cuda.Stream()
    res = {"lib": a.lib or "librt_mi355x.so", "inflight": a.inflight, "rays": a.rays, "items": a.items, "scene": a.scene, "view": a.view, "resolution": [w, h], "frames": a.frames, "per_n": {}}
    for n in [int(x) for x in a.ranks.split(",")]:
        npk = R.packed_pixels(w, h, n)
        rect = np.zeros(4, np.int32)
        _lib.call("rt_frame_rect", cam._h, None, 0, n, _lib.ptr(rect))
        ranks = []
        for r in range(n):
            bufs = [torch.zeros(npk, dtype=torch.int32, device="cuda:0") for _ in range(max(1, a.inflight))]
            loop = R.FrameLoop(cam, bufs, tile=(n, r), render_stream=st.cuda_stream,
                               event_every=1 if a.inflight <= 1 else 8, inflight=a.inflight)
            loop.run(20)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ms, cnt, host = loop.run(a.frames)
            period = 1e3 * (time.perf_counter() - t0) / a.frames
            if a.inflight > 1:
                ms = period  # the rank's frame period with frames overlapping
            send = int(_lib.lib().rt_rect_pixels(w, h, n, r, _lib.ptr(rect))) * 4 if r else 0
            ranks.append({"rank": r, "render_ms": round(ms, 5), "period_ms": round(period, 5), "host_us_per_frame": round(1e3 * host / a.frames, 2),
                          "rays_per_wave": cam.get_option(_lib.RT_OPT_RAYS_USED), "send_bytes": send})
        worst = max(x["render_ms"] for x in ranks)
        if a.stamps:
            r = max(range(n), key=lambda q: ranks[q]["render_ms"])
            ranks[r]["waves"] = wave_stamps(cam, _lib, R, torch, st, n, r, npk)
        res["per_n"][str(n)] = {"ranks": ranks, "max_render_ms": worst,
                                "render_bound_fps": round(1e3 / worst, 1) if worst else None,
                                "rect": [int(v) for v in rect]}
        print(f"N={n}: max render {worst:.4f} ms -> <= {1e3 / worst:.0f} FPS; per rank "
              f"{[x['render_ms'] for x in ranks]}", flush=True)
    if a.out:
        with open(a.out, "w") as fp:
            json.dump(res, fp, indent=1)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
