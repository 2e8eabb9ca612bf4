"""Diagnostic: where does a KD frame spend its time?  (GPU; not a test.)

Times the full kernel, the no-traversal variant (ray generation + root test
+ shading only) and records per-wave start/end clocks (s_memrealtime,
100 MHz) with each wave's maximum visit count.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from cpp_cuda_raytracer_dev_amd import _lib, raytracer as R
    from tests import helpers as H
    name = sys.argv[1] if len(sys.argv) > 1 else "dragon"
    w, h = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1920, 1080)
    kernel = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    rays = int(sys.argv[5]) if len(sys.argv) > 5 else 32
    order = int(sys.argv[6]) if len(sys.argv) > 6 else 2
    items = int(sys.argv[7]) if len(sys.argv) > 7 else 2
    extra = int(sys.argv[8]) if len(sys.argv) > 8 else 0  # extra debug bits (e.g. 1024: one-level iterations)
    s = H.GpuScene(name, w, h, kernel=kernel, tile_order=order, rays=rays, items=items)
    out = torch.zeros(w * h, dtype=torch.int32, device="cuda:0")
    st = torch.cuda.Stream()

    def timed(n=50):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(5):
            s.cam.render_into(out, stream=st.cuda_stream)
        e0.record(st)
        for _ in range(n):
            s.cam.render_into(out, stream=st.cuda_stream)
        e1.record(st)
        st.synchronize()
        return e0.elapsed_time(e1) / n

    s.cam.set_option(_lib.RT_OPT_DEBUG, extra)
    res = {"scene": name, "w": w, "h": h, "kernel": kernel, "rays": rays, "items": items, "debug": extra,
           "full_ms": timed()}
    s.cam.set_option(_lib.RT_OPT_DEBUG, 1 | extra)
    res["no_traversal_ms"] = timed()
    s.cam.set_option(_lib.RT_OPT_DEBUG, 2 | extra)
    res["with_stamps_ms"] = timed(5)
    nw = ((w + 7) // 8) * ((h + 7) // 8) * (64 // rays) * 2
    buf = np.zeros(3 * nw, np.uint64)
    got = _lib.lib().rt_camera_debug_read(s.cam._h, _lib.ptr(buf), len(buf))
    rec = buf[:got].reshape(-1, 3).astype(np.int64)
    rec = rec[rec[:, 1] > 0]
    t0 = rec[:, 0].min()
    start, end = (rec[:, 0] - t0) * 10e-3, (rec[:, 1] - t0) * 10e-3  # us
    vis, popped = rec[:, 2] & 0xFFFFFFFF, rec[:, 2] >> 32  # pool iterations, items popped
    coarse = vis == 0xFFFFFFFF  # k_coarse_kd3 waves (whole wave: its groups)
    if coarse.any():
        cd = end[coarse] - start[coarse]
        res["coarse_waves"] = int(coarse.sum())
        res["coarse_dur_us_p50_p99_max"] = [float(np.percentile(cd, q)) for q in (50, 99, 100)]
        res["coarse_start_us_min_max"] = [float(start[coarse].min()), float(start[coarse].max())]
        res["coarse_end_us_max"] = float(end[coarse].max())
        res["fine_start_us_min"] = float(start[~coarse].min())
    start, end, vis, popped = start[~coarse], end[~coarse], vis[~coarse], popped[~coarse]
    dur = end - start
    res["span_us"] = float(end.max())
    res["waves"] = int(len(rec))
    res["iters_total"] = int(vis[vis != 0xFFFFFFFF].sum())
    res["items_total"] = int(popped[vis != 0xFFFFFFFF].sum())
    res["wave_us_total"] = float(dur.sum())
    heavy = vis > 1
    res["heavy_waves"] = int(heavy.sum())
    for tag, m in (("light", ~heavy), ("heavy", heavy)):
        if m.any():
            res[f"{tag}_dur_us_p50_p99_max"] = [float(np.percentile(dur[m], q)) for q in (50, 99, 100)]
            res[f"{tag}_start_us_max"] = float(start[m].max())
            res[f"{tag}_end_us_max"] = float(end[m].max())
    if heavy.any():
        k = np.argmax(dur)
        res["longest_wave"] = {"dur_us": float(dur[k]), "visits": int(vis[k]), "start_us": float(start[k])}
        res["us_per_visit_longest"] = float(dur[k] / max(vis[k], 1))
        res["us_per_visit_median_heavy"] = float(np.median(dur[heavy] / np.maximum(vis[heavy], 1)))
        res["longest_wave"]["items"] = int(popped[k])
        res["items_per_iter_heavy_p10_p50_p90"] = [float(np.percentile(popped[heavy] / np.maximum(vis[heavy], 1), q))
                                                   for q in (10, 50, 90)]
        top = np.argsort(-dur)[:200]
        res["items_per_iter_200_longest"] = float(popped[top].sum() / max(vis[top].sum(), 1))
        res["iters_200_longest_mean"] = float(vis[top].mean())
    # when do light waves finish vs heavy waves start
    res["time_all_light_done_us"] = float(end[~heavy].max()) if (~heavy).any() else None
    print(json.dumps(res))


if __name__ == "__main__":
    main()
