#!/usr/bin/env python3
"""Host cost per frame of the moving-object path, split: the Python input
tick + transform, render_into with the same transform (cached launch
geometry), and render_into with a new transform each frame (launch geometry,
fine grid and tile order recomputed).

    python tools/host_cost.py [--frames 300]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--keys", default="R+W.Q.T.W")
    a = ap.parse_args()
    import torch
    from cpp_cuda_raytracer_dev_amd import raytracer as R
    import bench
    pts, leafs, nodes, _ = bench.build_scene("dragon")
    t = R.Trixel(len(pts), pts)
    t.set_kd_nodes(nodes)
    cam = R.Camera.default(1920, 1080)
    obj = R.Object(t)
    cam.add_object(obj)
    masks = bench.key_masks(a.keys)
    out = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda:0")
    st = torch.cuda.Stream()
    xfs = []
    t0 = time.perf_counter()
    for i in range(a.frames):
        obj.key_tick(masks[i % len(masks)])
        xfs.append(obj.quat.xform())
    tick = (time.perf_counter() - t0) / a.frames
    for xf in xfs[:20]:
        cam.render_into(out, xform=xf, stream=st.cuda_stream)
    st.synchronize()
    res = {"tick_us": tick * 1e6}
    from cpp_cuda_raytracer_dev_amd import _lib
    runs = [("same_xform", [xfs[0]] * a.frames), ("same_xform_mid", [xfs[len(xfs) // 2]] * a.frames),
            ("same_xform_last", [xfs[-1]] * a.frames), ("new_xform", xfs),
            ("alternate_2", [xfs[i % 2] for i in range(a.frames)])]
    for order in (1, 2, 3):
        runs.append((f"new_xform_order{order}", xfs))
    for name, seq in runs:
        if name.startswith("new_xform_order"):
            cam.set_option(_lib.RT_OPT_TILE_ORDER, int(name[-1]))
        st.synchronize()
        t0 = time.perf_counter()
        for xf in seq:
            cam.render_into(out, xform=xf, stream=st.cuda_stream)
        host = (time.perf_counter() - t0) / a.frames
        st.synchronize()
        res[name + "_host_us"] = host * 1e6
        res[name + "_period_us"] = (time.perf_counter() - t0) / a.frames * 1e6
    print(res, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
