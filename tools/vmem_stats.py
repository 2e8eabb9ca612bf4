#!/usr/bin/env python3
"""Record-load statistics of kernel 3's pool walks (verdict r05 item 1): per
walk form, live lanes per record load against distinct records and lines,
and the vector memory path's cycles by tools/ubench_l1.hip's model, from a
diagnostic build of the library (-DRT_VMEM_STATS=1; rt_kernels_impl.h
vmem_stat) and debug bit 16384.

    python -m cpp_cuda_raytracer_dev_amd.build --variant vstat --defs=-DRT_VMEM_STATS=1
    python tools/vmem_stats.py tools/variants/lib_vstat.so [--scene knot] [--width 1920 --height 1080]
        [--frames 4] [--rays 0] [--out profiles/r06/vmem_stats_knot.json]

Forms: 0 a single-slot pop (<= 64 items), 1 / 2 slot 0 / slot 1 of a
two-slot pop, 3 a two-level iteration.  A record group is four dwordx4 wave
loads (a 64-B record per lane).  model_cycles_per_load = sum over the 16
lane quads of max(1, distinct 128-B lines its loading lanes touch): what one
wave load costs the CU's address / data units (ubench_l1: 16 cycles when
every quad touches one line, 64 when every lane touches its own).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
FORMS = ["single-slot pop", "two-slot pop, slot 0", "two-slot pop, slot 1", "two-level iteration"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--scene", default="knot")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--rays", type=int, default=0)
    ap.add_argument("--shadow", action="store_true")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from cpp_cuda_raytracer_dev_amd import _lib
    _lib.LIB_PATH = os.path.abspath(a.lib)
    import numpy as np
    from cpp_cuda_raytracer_dev_amd import raytracer as R, scenes
    v, arity, idx = scenes.mesh_arrays(a.scene)
    pts, _, leafs = R.assemble_mesh(v, scenes.faces_of(arity, idx))
    trixel = R.Trixel(len(pts), pts)
    trixel.set_kd_nodes(R.kd_build(leafs))
    kw = scenes.view(a.scene, "default")
    cam = R.Camera(a.width, a.height, R.film_w(a.width, a.height), np.float32(.024), np.float32(.055), *kw["pos"],
                   *kw["look_at"], 0.0, 1.0, 0.0)
    cam.set_option(_lib.RT_OPT_KERNEL, 3)
    cam.set_option(_lib.RT_OPT_RAYS, a.rays)
    obj = R.Object(trixel)
    cam.add_object(obj)
    flags = R.RT_FLAG_SHADOW if a.shadow else 0
    # settle the cost order (tile order 3) with the statistics off, then count
    for _ in range(40):
        obj.render(cam, mode=0, flags=flags)
    cam.set_option(_lib.RT_OPT_DEBUG, 16384)
    for _ in range(a.frames):
        obj.render(cam, mode=0, flags=flags)
    raw = np.zeros(32, np.uint64)
    got = _lib.lib().rt_camera_debug_read(cam._h, _lib.ptr(raw), len(raw))
    assert got == 32, got
    out = {"scene": a.scene, "resolution": [a.width, a.height], "frames": a.frames, "shadow": a.shadow,
           "rays_per_wave": cam.get_option(_lib.RT_OPT_RAYS_USED), "fast": cam.get_option(_lib.RT_OPT_FAST_USED),
           "forms": {}}
    tot_live = tot_cycles = 0
    for f, name in enumerate(FORMS):
        g, live, load, qc, drec, dline = (int(x) for x in raw[6 * f:6 * f + 6])
        if not g:
            continue
        tot_live += live
        tot_cycles += 4 * qc
        out["forms"][name] = {
            "record_groups_per_frame": g / a.frames, "live_items_per_frame": live / a.frames,
            "live_lanes_per_group": live / g, "loading_lanes_per_group": load / g,
            "distinct_records_per_group": drec / g, "distinct_lines_per_group": dline / g,
            "model_cycles_per_load": qc / g, "model_cycles_per_visit": 4 * qc / live if live else None,
            "ideal_cycles_per_load": 16.0}
    out["model_cycles_per_visit_all"] = tot_cycles / tot_live if tot_live else None
    out["model_cycles_per_frame_per_cu"] = tot_cycles / a.frames / 256.0
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as fp:
            json.dump(out, fp, indent=1)
    cam.close()
    obj.motion.close()
    trixel.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
