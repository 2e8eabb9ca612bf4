"""Regenerate tests/golden/golden_frames.npz (committed fixtures).

Small frames are rendered by the independent numpy restatement
(oracle/np_oracle.py); the larger ones by the C restatement
(oracle/oracle.c), recorded as SHA-256 of the u32 frame and the int64 hit
buffer plus a full-width crop.  The two restatements agree bit-for-bit on
every small frame (tests/test_oracle_crosscheck.py), which is how the C
oracle is pinned: the reference itself has no fixtures and cannot be run
here.
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from cpp_cuda_raytracer_dev_amd import scenes  # noqa: E402
from oracle import _oracle as O, np_oracle as N  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden_frames.npz")
SMALL = [("dump_test", 64, 36), ("tester", 80, 45), ("dump", 48, 27)]
LARGE = [("tester", 320, 180, 0), ("tester", 320, 180, 1), ("rabbit_70k", 960, 540, 0), ("dump", 320, 180, 0)]
# shadow-ray frames (RT_FLAG_SHADOW): numpy full frames,
# C-oracle hashes + counters.  `--shadow` adds only these keys to the file.
SHADOW_SMALL = [("dump", 40, 24), ("rabbit_70k", 64, 36)]
SHADOW_LARGE = [("rabbit_70k", 960, 540), ("dump", 320, 180)]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def shadow_keys(out):
    for name, w, h in SHADOW_SMALL:
        v, a, ix = scenes.fixture_mesh(name)
        pts, boxes = N.assemble(v, a, ix)
        argb, hit = N.render(pts, N.build_kd(boxes), N.camera(w, h), 0, shadow=True)
        out[f"{name}_{w}x{h}_shadow_argb"] = argb
        out[f"{name}_{w}x{h}_shadow_hit"] = hit
        print(name, w, h, "shadow", (hit >= 0).sum(), ((argb == 0) & (hit >= 0)).sum(), flush=True)
    for name, w, h in SHADOW_LARGE:
        v, a, ix = scenes.fixture_mesh(name)
        pts, lf = O.assemble(v, a, ix)
        s = O.Scene(pts, O.default_rad(len(pts)), O.build_kd(lf), O.camera(w, h))
        argb, hit, cnt = s.render(0, shadow=True)
        key = f"{name}_{w}x{h}_shadow"
        out[key + "_argb_sha"] = np.array(sha(argb))
        out[key + "_counters"] = cnt
        print(key, ((argb == 0) & (hit >= 0)).sum(), cnt, flush=True)


def main():
    if "--shadow" in sys.argv:
        with np.load(OUT, allow_pickle=False) as z:
            out = {k: z[k] for k in z.files}
        shadow_keys(out)
        np.savez_compressed(OUT, **out)
        print("updated", OUT)
        return 0
    out = {}
    for name, w, h in SMALL:
        v, a, ix = scenes.fixture_mesh(name)
        pts, boxes = N.assemble(v, a, ix)
        nodes = N.build_kd(boxes)
        cam = N.camera(w, h)
        for mode in (0, 1):
            argb, hit = N.render(pts, nodes, cam, mode)
            out[f"{name}_{w}x{h}_m{mode}_argb"] = argb
            out[f"{name}_{w}x{h}_m{mode}_hit"] = hit
            print(name, w, h, mode, (hit >= 0).sum(), flush=True)
    for name, w, h, mode in LARGE:
        v, a, ix = scenes.fixture_mesh(name)
        pts, lf = O.assemble(v, a, ix)
        nodes = O.build_kd(lf) if mode == 0 else None
        s = O.Scene(pts, O.default_rad(len(pts)), nodes, O.camera(w, h))
        argb, hit, cnt = s.render(mode)
        key = f"{name}_{w}x{h}_m{mode}"
        out[key + "_argb_sha"] = np.array(sha(argb))
        out[key + "_hit_sha"] = np.array(sha(hit))
        out[key + "_counters"] = cnt
        r0 = h // 2 - 4
        out[key + "_crop_rows"] = np.array([r0, r0 + 8])
        out[key + "_crop_argb"] = argb.reshape(h, w)[r0:r0 + 8].copy()
        out[key + "_crop_hit"] = hit.reshape(h, w)[r0:r0 + 8].copy()
        print(key, (hit >= 0).sum(), cnt, flush=True)
    shadow_keys(out)
    np.savez_compressed(OUT, **out)
    print("wrote", OUT)
    return 0


if __name__ == "__main__":
    sys.exit(main())
