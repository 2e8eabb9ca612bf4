"""The rectangle gather's sizes and assembly time (one GPU): rt_frame_rect for
N = 1, 2, 4, 8 on the dragon stand-in at 1920x1080, the bytes each peer sends,
and the rank-0 assembly kernels timed with HIP events.

    python tools/rect_info.py
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from cpp_cuda_raytracer_dev_amd import _lib, raytracer as R
    from tests import helpers as H
    w, h = 1920, 1080
    s = H.GpuScene("dragon", w, h)
    s.render(0)
    out = {"scene": "dragon stand-in", "resolution": [w, h], "frame_bytes": w * h * 4, "ranks": {}}
    dev = torch.device("cuda:0")
    for n in (1, 2, 4, 8):
        rect = np.zeros(4, np.int32)
        _lib.call("rt_frame_rect", s.cam._h, None, 0, n, _lib.ptr(rect))
        counts = [int(_lib.lib().rt_rect_pixels(w, h, n, r, _lib.ptr(rect))) for r in range(n)]
        npk = R.packed_pixels(w, h, n)
        local = torch.zeros(npk, dtype=torch.int32, device=dev)
        peers = torch.zeros(max(1, (n - 1) * npk), dtype=torch.int32, device=dev)
        frame = torch.zeros(w * h, dtype=torch.int32, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(10):
            _lib.call("rt_unpack_rect", 0, w, h, n, _lib.ptr(rect), _lib.ptr(local), _lib.ptr(peers), _lib.ptr(frame),
                      None)
        e0.record()
        for _ in range(100):
            _lib.call("rt_unpack_rect", 0, w, h, n, _lib.ptr(rect), _lib.ptr(local), _lib.ptr(peers), _lib.ptr(frame),
                      None)
        e1.record()
        torch.cuda.synchronize()
        out["ranks"][n] = {"rect_x0_x1_b0_b1": [int(v) for v in rect],
                           "peer_send_bytes": [4 * c for c in counts[1:]],
                           "full_band_bytes_per_peer": 4 * npk,
                           "unpack_rect_us": round(e0.elapsed_time(e1) * 10, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
