"""Diagnostic (GPU; not a test): coop / split tile counts after N frames for
identity and moved poses, debug 0 / 4096, rays auto / 8 / 16."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rot_y(deg, t=(0.0, 0.0, 0.0)):
    a = np.deg2rad(np.float64(deg))
    c, s = np.float32(np.cos(a)), np.float32(np.sin(a))
    return np.array([[c, 0, s, t[0]], [0, 1, 0, t[1]], [-s, 0, c, t[2]]], np.float32).reshape(12)


def main():
    import torch
    from cpp_cuda_raytracer_dev_amd import _lib, raytracer as R
    from tests import helpers as H
    w, h = 960, 540
    out = []
    for pose in ("identity", "rot3"):
        xf = rot_y(0.0) if pose == "identity" else rot_y(3.0)
        for debug in (0, 4096):
            for rays in (0, 8, 16):
                s = H.GpuScene("dragon", w, h, rays=rays, debug=debug or None)
                o = torch.zeros(w * h, dtype=torch.int32, device="cuda:0")
                st = torch.cuda.Stream()
                seq = []
                for k in range(48):
                    s.cam.render_into(o, xform=xf, stream=st.cuda_stream)
                    st.synchronize()
                    if k % 8 == 7:
                        seq.append((s.cam.get_option(_lib.RT_OPT_COOP_USED), s.cam.get_option(_lib.RT_OPT_SPLIT_USED),
                                    s.cam.get_option(_lib.RT_OPT_RAYS_USED)))
                out.append({"pose": pose, "debug": debug, "rays": rays, "coop_split_rays_every8": seq})
                print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
