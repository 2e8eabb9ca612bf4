#!/usr/bin/env python3
"""Diagnostic (GPU; not a test): where one pool iteration of kernel 3 spends
its time.  Needs the stamps build (tools/build_variants.sh
stamps:"-DRT_ITER_STAMPS=1").  Renders solo frames with debug bits 2 | 128,
reads each unit's per-iteration shader-clock stamps and prints, for the
heaviest units (the frame's chain) and for all units, the mean cycles of the
phases:  pop (items from LDS) | record wait | item 0 visit + push |
item 1 visit + push, by pool size.

    python tools/diag_iters.py tools/variants/lib_stamps.so [scene W H rays]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from cpp_cuda_raytracer_dev_amd import _lib
    _lib.LIB_PATH = os.path.abspath(sys.argv[1])
    import torch
    from tests import helpers as H
    name = sys.argv[2] if len(sys.argv) > 2 else "knot"
    w, h = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (1920, 1080)
    rays = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    s = H.GpuScene(name, w, h, rays=rays)
    out = torch.zeros(w * h, dtype=torch.int32, device="cuda:0")
    for _ in range(40):  # the cost order settles
        s.cam.render_into(out)
    torch.cuda.synchronize()
    s.cam.set_option(_lib.RT_OPT_DEBUG, 2 | 128)
    s.cam.render_into(out)
    torch.cuda.synchronize()
    off = s.cam.get_option(102)
    K = 96
    buf = np.zeros(off + (off // 3) * 4 * K + 16, np.uint64)
    got = _lib.lib().rt_camera_debug_read(s.cam._h, _lib.ptr(buf), len(buf))
    buf = buf[:got]
    per = buf[:off].reshape(-1, 3).astype(np.int64)
    st = buf[off:off + (off // 3) * 4 * K].reshape(-1, K, 4).astype(np.int64)
    iters = per[:, 2] & 0xFFFFFFFF
    live = (per[:, 1] > 0) & (iters > 0) & (iters != 0xFFFFFFFF)
    idx = np.nonzero(live)[0]
    res = {"scene": name, "w": w, "h": h, "rays_used": s.cam.get_option(_lib.RT_OPT_RAYS_USED), "units": int(len(idx))}

    def phases(sel_units, nmax=K):
        rows = []
        for u in sel_units:
            n = int(min(iters[u], nmax))
            q = st[u, :n]
            d1, d2 = q[:, 1] & 0xFFFFFFFF, q[:, 1] >> 32
            d3, d4 = q[:, 2] & 0xFFFFFFFF, q[:, 2] >> 32
            take, pool = q[:, 3] & 0xFFFFFFFF, q[:, 3] >> 32
            gap = np.r_[q[1:, 0] - (q[:-1, 0] + d1[:-1] + d2[:-1] + d3[:-1] + d4[:-1]), 0]
            rows.append(np.stack([d1, d2, d3, d4, gap, take, pool], 1))
        return np.concatenate(rows) if rows else np.zeros((0, 7))

    heavy = idx[np.argsort(-iters[idx])][:32]
    res["heaviest_iters"] = [int(iters[u]) for u in heavy[:8]]
    names = ["pop", "record_wait", "visit_push_0", "visit_push_1", "loop_gap"]
    for label, sel in (("heaviest32", heavy), ("all", idx)):
        P = phases(sel)
        if not len(P):
            continue
        res[label] = {"iterations": int(len(P)),
                      "mean_cycles": {k: round(float(P[:, i].mean()), 1) for i, k in enumerate(names)},
                      "mean_take": round(float(P[:, 5].mean()), 1)}
        byt = {}
        for lo, hi in ((1, 16), (16, 64), (64, 128), (128, 129)):
            m = (P[:, 5] >= lo) & (P[:, 5] < hi)
            if m.any():
                byt[f"take_{lo}_{hi - 1}"] = {"n": int(m.sum()),
                                             **{k: round(float(P[m, i].mean()), 1) for i, k in enumerate(names)}}
        res[label]["by_take"] = byt
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
