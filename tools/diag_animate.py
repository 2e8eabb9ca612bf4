#!/usr/bin/env python3
"""Diagnose a moving-object frame sequence frame by frame: one input tick,
one kernel-3 render, a device synchronisation and the error word after each,
printing the frame's launch facts; stops at the first failure.

    python tools/diag_animate.py [--keys R+W.Q.T.W] [--frames 600] [--every 1]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", default="R+W.Q.T.W")
    ap.add_argument("--frames", type=int, default=600)
    ap.add_argument("--rays", type=int, default=0)
    ap.add_argument("--tile-order", type=int, default=3)
    ap.add_argument("--sync-every", type=int, default=1)
    a = ap.parse_args()
    import torch
    from cpp_cuda_raytracer_dev_amd import _lib, raytracer as R
    import bench
    pts, leafs, nodes, _ = bench.build_scene("dragon")
    t = R.Trixel(len(pts), pts)
    t.set_kd_nodes(nodes)
    cam = R.Camera.default(1920, 1080)
    obj = R.Object(t)
    cam.add_object(obj)
    cam.set_option(_lib.RT_OPT_RAYS, a.rays)
    cam.set_option(_lib.RT_OPT_TILE_ORDER, a.tile_order)
    masks = bench.key_masks(a.keys)
    out = torch.zeros(1920 * 1080, dtype=torch.int32, device="cuda:0")
    st = torch.cuda.Stream()
    t0 = time.time()
    for i in range(a.frames):
        obj.key_tick(masks[i % len(masks)])
        xf = obj.quat.xform()
        cam.render_into(out, xform=xf, mode=0, stream=st.cuda_stream)
        if (i + 1) % a.sync_every == 0:
            st.synchronize()
            err = cam.device_error(reset=True)
            print(f"frame {i}: rays {cam.get_option(_lib.RT_OPT_RAYS_USED)} t=({xf[3]:.4f},{xf[7]:.4f},{xf[11]:.4f}) "
                  f"err {err} {time.time() - t0:.2f}s", flush=True)
            if err:
                return 3
    st.synchronize()
    print("done", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
