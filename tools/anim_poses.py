#!/usr/bin/env python3
"""Per-pose cost of a moving-object run (design tool, not a test): for the
poses `bench.py --animate KEYS` renders, each pose's solo kernel time (one
frame alone, HIP events on the render stream), its interior visits and root
passes (a counting render), and which walk it took (RT_OPT_FAST_USED), beside
the static pose through the untranslated walk.

    python tools/anim_poses.py [--scene dragon] [--keys R+W.Q.T.W] [--frames 1000] [--every 10]
        [--out profiles/r06/anim_poses.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="dragon")
    ap.add_argument("--keys", default="R+W.Q.T.W")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--every", type=int, default=10)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import numpy as np
    import torch
    from cpp_cuda_raytracer_dev_amd import _lib, raytracer as R, scenes
    import bench
    dev = torch.device("cuda", 0)
    pts, leafs, nodes, _ = bench.build_scene(a.scene)
    trixel = R.Trixel(len(pts), pts, device=0)
    trixel.set_kd_nodes(nodes)
    kw = scenes.view(a.scene, "default")
    cam = R.Camera(a.width, a.height, R.film_w(a.width, a.height), np.float32(.024), np.float32(.055), *kw["pos"],
                   *kw["look_at"], 0.0, 1.0, 0.0, device=0)
    cam.set_option(_lib.RT_OPT_KERNEL, 3)
    obj = R.Object(trixel)
    cam.add_object(obj)
    argb = torch.zeros(a.width * a.height, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(device=dev)
    sptr = stream.cuda_stream

    def measure(xf):
        for _ in range(3):
            cam.render_into(argb, xform=xf, stream=sptr)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(a.reps):
            cam.render_into(argb, xform=xf, stream=sptr)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        us = e0.elapsed_time(e1) * 1000.0 / a.reps
        fast = cam.get_option(_lib.RT_OPT_FAST_USED)
        cam.set_option(_lib.RT_OPT_KERNEL, 2)  # the reference's DFS order counts (bench.py)
        cam.render_into(argb, xform=xf, flags=R.RT_FLAG_COUNT, stream=sptr)
        torch.cuda.synchronize(dev)
        c = cam.counters(reset=True)
        cam.set_option(_lib.RT_OPT_KERNEL, 3)
        return us, fast, [int(x) for x in c]

    out = {"scene": a.scene, "keys": a.keys, "resolution": [a.width, a.height], "reps": a.reps, "poses": []}
    us, fast, c = measure(None)
    out["static"] = {"us": round(us, 2), "fast": fast, "counters": c}
    print("static", out["static"], flush=True)
    masks = bench.key_masks(a.keys)
    mo = R.ObjectMotion(cam.pos, cam.o_prop["n"], cam.o_prop["u"], cam.cam_speed)
    for i in range(a.frames):
        mo.tick(masks[i % len(masks)])
        if i % a.every:
            continue
        xf = np.asarray(mo.xform(), np.float32).reshape(12)
        us, fast, c = measure(xf)
        out["poses"].append({"i": i, "us": round(us, 2), "fast": fast, "counters": c,
                             "offset": [float(xf[3]), float(xf[7]), float(xf[11])]})
        print(i, round(us, 2), fast, c, flush=True)
    mo.close()
    t = np.array([p["us"] for p in out["poses"]])
    nint = np.array([p["counters"][0] for p in out["poses"]], np.float64)
    out["summary"] = {"mean_us": float(t.mean()), "median_us": float(np.median(t)), "max_us": float(t.max()),
                      "mean_interior_visits": float(nint.mean()),
                      "ns_per_interior_visit_poses": float(t.sum() * 1e3 / nint.sum()),
                      "ns_per_interior_visit_static": out["static"]["us"] * 1e3 / max(1, out["static"]["counters"][0]),
                      "fast_all": all(p["fast"] & 1 for p in out["poses"])}
    print(json.dumps(out["summary"]))
    if a.out:
        with open(a.out, "w") as fp:
            json.dump(out, fp, indent=1)
    cam.close()
    obj.motion.close()
    trixel.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
