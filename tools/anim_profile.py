#!/usr/bin/env python3
"""Frame time along a key sequence (the far-along
moving-object frame): the dragon at 1920x1080 driven by `--keys` for
`--frames` ticks, rendered one frame at a time through rt_run_frames with the
sequence's own poses, in batches of `--batch` frames between one pair of HIP
events.  Per batch: the mean frame time and the mean coverage (an untimed
counting render of every `--count-every`-th pose).

    python tools/anim_profile.py [--keys R+W.Q.T.W] [--frames 10000] [--batch 500] [--start 0] [--out file.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", default="R+W.Q.T.W")
    ap.add_argument("--scene", default="dragon")
    ap.add_argument("--frames", type=int, default=10000)
    ap.add_argument("--batch", type=int, default=500)
    ap.add_argument("--start", type=int, default=0, help="first tick rendered (the poses before it are only ticked)")
    ap.add_argument("--count-every", type=int, default=25)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch
    import bench
    from cpp_cuda_raytracer_dev_amd import _lib, scenes, raytracer as R
    w, h = a.width, a.height
    pts, leafs, nodes, _ = bench.build_scene(a.scene)
    trixel = R.Trixel(len(pts), pts, device=0)
    trixel.set_kd_nodes(nodes)
    kw = scenes.view(a.scene, "default")
    cam = R.Camera(w, h, R.film_w(w, h), np.float32(.024), np.float32(.055), *kw["pos"], *kw["look_at"],
                   0.0, 1.0, 0.0, device=0)
    cam.set_option(_lib.RT_OPT_KERNEL, 3)
    cam.set_option(_lib.RT_OPT_TILE_ORDER, 3)
    obj = R.Object(trixel)
    cam.add_object(obj)
    masks = bench.key_masks(a.keys)
    mo = R.ObjectMotion(cam.pos, cam.o_prop["n"], cam.o_prop["u"], cam.cam_speed)
    poses = []
    for i in range(a.frames):
        mo.tick(masks[i % len(masks)])
        poses.append(np.asarray(mo.xform(), np.float32).reshape(12))
    mo.close()
    poses = np.stack(poses)
    out = torch.zeros(w * h, dtype=torch.int32, device="cuda:0")
    st = torch.cuda.Stream()
    rows = []
    for b0 in range(a.start, a.frames, a.batch):
        b1 = min(a.frames, b0 + a.batch)
        # coverage of this batch's poses (untimed counting renders)
        hits = []
        for i in range(b0, b1, a.count_every):
            cam.render_into(out, xform=poses[i], flags=R.RT_FLAG_COUNT, stream=st.cuda_stream)
            st.synchronize()
            hits.append(float(cam.counters(reset=True)[3]))
        loop = R.FrameLoop(cam, [out], mode=0, render_stream=st.cuda_stream, event_every=0, inflight=1,
                           xforms=poses[b0:b1])
        loop.run(b1 - b0)  # settles the cost order / held region for these poses
        loop.seq.value = 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        loop.run(b1 - b0)
        e1.record(st)
        st.synchronize()
        us = 1e3 * e0.elapsed_time(e1) / (b1 - b0)
        err = cam.device_error(reset=True)
        rows.append({"ticks": [b0 + 1, b1], "us_per_frame": round(us, 2),
                     "coverage": round(float(np.mean(hits)) / (w * h), 5), "device_err": err})
        print(json.dumps(rows[-1]), flush=True)
    res = {"scene": a.scene, "keys": a.keys, "frames": a.frames, "w": w, "h": h,
           "build_id": _lib.build_id(), "batches": rows}
    if a.out:
        with open(a.out, "w") as fp:
            json.dump(res, fp, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
