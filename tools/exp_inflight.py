#!/usr/bin/env python3
"""Frames in flight on one GPU: consecutive frames of the same view rendered
on 1 or 2 streams (each into its own buffer), for several ways of getting the
second stream: torch's pool, a high-priority torch stream, and HIP streams
with a full CU mask (hipExtStreamCreateWithCUMask, a dedicated hardware
queue).  Prints frames/s per variant and checks every buffer against the
single-stream frame.

    python tools/exp_inflight.py [--frames 2000] [--width 1920 --height 1080] [--scene dragon]
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=2000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--scene", default="dragon")
    ap.add_argument("--view", default="default")
    ap.add_argument("--variants", default="one,pool2,prio,cumask2,cumask3")
    a = ap.parse_args()
    import torch
    from cpp_cuda_raytracer_dev_amd import _lib, raytracer as R, scenes
    import bench
    pts, leafs, nodes, _ = bench.build_scene(a.scene)
    w, h = a.width, a.height
    t = R.Trixel(len(pts), pts)
    t.set_kd_nodes(nodes)
    kw = scenes.view(a.scene, a.view)
    cam = R.Camera(w, h, R.film_w(w, h), np.float32(.024), np.float32(.055), *kw["pos"], *kw["look_at"], 0.0, 1.0, 0.0)
    cam.add_object(R.Object(t))
    hip = ctypes.CDLL("libamdhip64.so")
    cu = int(torch.cuda.get_device_properties(0).multi_processor_count)

    def cumask_stream():
        s = ctypes.c_void_p()
        words = (cu + 31) // 32
        mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
        assert rc == 0, rc
        return s.value

    ref = torch.zeros(w * h, dtype=torch.int32, device="cuda:0")
    st0 = torch.cuda.Stream()
    for _ in range(40):
        cam.render_into(ref, stream=st0.cuda_stream)
    st0.synchronize()
    res = {}
    for v in a.variants.split(","):
        if v == "one":
            ss = [st0.cuda_stream]
        elif v == "pool2":
            ss = [st0.cuda_stream, torch.cuda.Stream().cuda_stream]
        elif v == "prio":
            ss = [st0.cuda_stream, torch.cuda.Stream(priority=-1).cuda_stream]
        elif v.startswith("cumask"):
            ss = [cumask_stream() for _ in range(int(v[6:]))]
        bufs = [torch.zeros(w * h, dtype=torch.int32, device="cuda:0") for _ in ss]
        for j in range(100):
            cam.render_into(bufs[j % len(ss)], stream=ss[j % len(ss)])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for j in range(a.frames):
            cam.render_into(bufs[j % len(ss)], stream=ss[j % len(ss)])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ok = all(torch.equal(b, ref) for b in bufs)
        err = cam.device_error(reset=True)
        res[v] = {"fps": round(a.frames / dt, 1), "us_per_frame": round(1e6 * dt / a.frames, 2), "frames_ok": ok, "err": err}
        print(v, res[v], flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
