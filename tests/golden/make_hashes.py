"""Regenerate tests/golden/frame_hashes.json (committed fixtures): full-frame
SHA-256 of the C oracle's u32 frame and int64 hit buffer, its visit counters
and pixel coverage, for every BASELINE config and bench view.

    python tests/golden/make_hashes.py [substring ...]   # only matching keys

The oracle (oracle/oracle.c) is the parity anchor: pinned by the numpy
restatement and hand KATs (tests/test_host_cpu.py), since the reference has
no fixtures and cannot run here.  The GPU tests and bench.py's
frame check compare the HIP path's full frames with these hashes.  Stand-in
meshes are generated with numpy (scenes.standin), so each entry records the
mesh's SHA-256: a host whose numpy produced other vertex bits regenerates the
frame with the oracle instead of trusting the hash.
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from cpp_cuda_raytracer_dev_amd import scenes  # noqa: E402
from oracle import _oracle as O  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "frame_hashes.json")

# (scene, w, h, mode, shadow, view)
FRAMES = [
    ("tester", 320, 180, 0, False, "default"),      # C1 (KD)
    ("tester", 320, 180, 1, False, "default"),      # C1 (flat)
    ("rabbit_70k", 960, 540, 1, False, "default"),  # C2: flat list, 3.6e10 tests
    ("rabbit_70k", 960, 540, 0, False, "default"),
    ("rabbit_70k", 1920, 1080, 0, False, "fill"),   # real mesh filling a 1080p frame
    ("dragon", 960, 540, 0, False, "default"),      # C3
    ("dragon", 1920, 1080, 0, False, "default"),    # C4 / the headline bench frame
    ("dragon", 1920, 1080, 0, True, "default"),
    ("dragon", 960, 540, 0, False, "fill"),         # README.md:19's ">= 90 % coverage" view
    ("dragon", 1920, 1080, 0, False, "fill"),
    ("happy", 1920, 1080, 0, True, "default"),
    ("happy", 3840, 2160, 0, False, "default"),
    ("happy", 3840, 2160, 0, True, "default"),      # C5
    ("big", 1920, 1080, 0, False, "default"),       # 3.1M triangles: a 22-level tree in kernel 3
    ("big", 1920, 1080, 0, True, "default"),
    ("knot", 960, 540, 0, False, "default"),       # the harder dragon-sized stand-in
    ("knot", 1920, 1080, 0, False, "default"),
    ("knot", 1920, 1080, 0, True, "default"),
]


def key_of(scene, w, h, mode, shadow, view):
    return f"{scene}_{w}x{h}_m{mode}" + ("_shadow" if shadow else "") + ("" if view == "default" else f"_{view}")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    only = sys.argv[1:]
    data = {"frames": {}, "meshes": {}}
    if os.path.exists(OUT):
        with open(OUT) as fp:
            data = json.load(fp)
    threads = int(os.environ.get("RT_ORACLE_THREADS", os.cpu_count() or 8))
    cache = {}
    for scene, w, h, mode, shadow, view in FRAMES:
        key = key_of(scene, w, h, mode, shadow, view)
        if only and not any(s in key for s in only):
            continue
        if scene not in cache:
            v, a, ix = scenes.mesh_arrays(scene)
            pts, lf = O.assemble(v, a, ix)
            t = time.perf_counter()
            nodes = O.build_kd(lf)
            cache[scene] = (pts, nodes)
            data["meshes"][scene] = scenes.mesh_sha(scene)
            print(f"{scene}: {len(pts)} triangles, oracle KD build {time.perf_counter() - t:.1f} s", flush=True)
        pts, nodes = cache[scene]
        cam = O.camera(w, h, **scenes.view(scene, view))
        s = O.Scene(pts, O.default_rad(len(pts)), nodes if mode == 0 else None, cam)
        t = time.perf_counter()
        argb, hit, cnt = s.render(mode, nthreads=threads, shadow=shadow)
        s.close()
        dt = time.perf_counter() - t
        data["frames"][key] = {
            "scene": scene, "w": w, "h": h, "mode": mode, "shadow": shadow, "view": view,
            "camera": scenes.view(scene, view),
            "mesh_sha": data["meshes"][scene],
            "argb_sha": sha(argb), "hit_sha": sha(hit),
            # interior visits, leaf visits, accepted hits, hit pixels, descents, max stack
            "counters": [int(x) for x in cnt],
            "hit_pixels": int((hit >= 0).sum()),
            "coverage": round(float((hit >= 0).mean()), 5),
            "shadowed_pixels": int(((argb == 0) & (hit >= 0)).sum()) if shadow else 0,
        }
        print(f"{key}: coverage {data['frames'][key]['coverage']:.4f} counters {data['frames'][key]['counters']} "
              f"({dt:.1f} s)", flush=True)
    data["generator"] = ("tests/golden/make_hashes.py: oracle/oracle.c (gcc -O3 -ffp-contract=off), "
                         "full frames, SHA-256 of the u32 frame and the int64 hit buffer")
    with open(OUT, "w") as fp:
        json.dump(data, fp, indent=1, sort_keys=True)
    print("wrote", OUT)
    return 0


if __name__ == "__main__":
    sys.exit(main())
