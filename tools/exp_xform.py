#!/usr/bin/env python3
"""Frame time of the dragon 1080p frame under fixed object transforms
(identity, a rotation, a translation, both), one frame in flight, so the
cost of the translated kernel instance and of the unfused far groups shows
apart from motion (no fine-grid change between frames).

    python tools/exp_xform.py [--frames 300]
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
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--scene", default="dragon")
    ap.add_argument("--tile-orders", default="3", help="comma list of RT_OPT_TILE_ORDER values")
    ap.add_argument("--debug", default="0", help="comma list of RT_OPT_DEBUG values (32: no device cost reorder)")
    ap.add_argument("--only", default="", help="comma list of pose names to run (default: all)")
    ap.add_argument("--holds", default="1", help="comma list: frames each pose of the moving sequence is held")
    ap.add_argument("--spin", type=float, default=0.01, help="rad per frame of the moving pose sequence")
    a = ap.parse_args()
    import torch
    from cpp_cuda_raytracer_dev_amd import _lib, raytracer as R, scenes
    v, ar, ix = scenes.mesh_arrays(a.scene)
    pts, n, leafs = R.assemble_mesh(v, scenes.faces_of(ar, ix))
    tri = R.Trixel(n, pts)
    tri.set_kd_nodes(R.kd_build(leafs))
    cam = R.Camera.default(1920, 1080)
    obj = R.Object(tri)
    cam.add_object(obj)
    c, s = np.cos(0.3), np.sin(0.3)
    poses = {
        "identity": [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0],
        "rotate_y": [c, 0, s, 0, 0, 1, 0, 0, -s, 0, c, 0],
        "translate": [1, 0, 0, 0.01, 0, 1, 0, -0.005, 0, 0, 1, 0.02],
        "rotate+translate": [c, 0, s, 0.01, 0, 1, 0, -0.005, -s, 0, c, 0.02],
    }
    # a moving object: rotate about y by `spin` per frame and drift, one pose per frame
    seq = []
    for k in range(64):
        ck, sk = np.cos(a.spin * k), np.sin(a.spin * k)
        seq.append([ck, 0, sk, 0.0002 * k, 0, 1, 0, 0, -sk, 0, ck, 0.0003 * k])
    for hold in [int(x) for x in a.holds.split(",")]:
        poses["moving" if hold == 1 else f"moving_hold{hold}"] = [x for x in seq for _ in range(hold)]
    if a.only:
        poses = {k: v for k, v in poses.items() if k in a.only.split(",")}
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    out = {}
    cases = [(o, d) for o in a.tile_orders.split(",") for d in a.debug.split(",")]
    for order, dbg in [(int(o), int(d)) for o, d in cases]:
      cam.set_option(_lib.RT_OPT_TILE_ORDER, order)
      cam.set_option(_lib.RT_OPT_DEBUG, dbg)
      for name0, xf in poses.items():
        name = f"{name0}/order{order}/debug{dbg}"
        xf = np.asarray(xf, np.float32)
        bufs = [torch.zeros(1920 * 1080, dtype=torch.int32, device=dev)]
        if xf.ndim == 2:
            loop = R.FrameLoop(cam, bufs, xforms=xf, render_stream=st.cuda_stream, event_every=0, inflight=1)
        else:
            loop = R.FrameLoop(cam, bufs, xform=xf, render_stream=st.cuda_stream, event_every=0, inflight=1)
        loop.run(50)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        loop.run(a.frames)
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.frames
        out[name] = {"us_per_frame": round(1e3 * ms, 2), "rays": cam.get_option(_lib.RT_OPT_RAYS_USED),
                     "err": cam.device_error(reset=True)}
        print(name, out[name], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
