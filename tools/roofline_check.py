#!/usr/bin/env python3
"""Recompute every configuration's roofline.frac from profiles/ alone
(VERDICT r03 item 1): the committed PMC entry (profiles/pmc_traffic.json:
HBM bytes per launch, VALU issue share, build id) and the rocprofv3
--kernel-trace --stats average of the same configuration's solo frames
(profiles/<round>/rocprof/<tag>_solo_kernel_stats.csv: the bench arguments
with --inflight 1, so every launch is one frame), against the bench line's
frac (profiles/<round>/bench/<tag>.json).

    python tools/roofline_check.py profiles/r04 [--out profiles/r04/roofline_check.md]

frac = max(L2-miss bytes / rocprof average / 8 TB/s, VALU issue share,
vector-memory (TD busy) share): the utilisation of the binding resource, as
bench.py computes it with its own kernel time (round 6 adds vmem_util, the
busy share of the texture data unit, and the traffic over the compulsory
scene + frame bytes).  A row agrees when the two are within 5 %.
"""
import argparse
import csv
import glob
import gzip
import json
import os

HBM = 8000.0  # GB/s
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bench_line(path):
    with open(path) as fp:
        lines = [ln for ln in fp if ln.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def stats_avg_us(path, kernel="k_trace_kd3"):
    with open(path) as fp:
        rows = [r for r in csv.DictReader(fp) if kernel in r["Name"]]
    if not rows:
        return None
    # the dominant instance (most total time)
    r = max(rows, key=lambda r: float(r["TotalDurationNs"]))
    return float(r["AverageNs"]) / 1e3, r["Name"][:60], int(r["Calls"])


def trace_per_frame_us(path, kernel="k_trace_kd3"):
    """Multi-frame launches in a kernel trace (the bench's own run): their
    total duration over the frames they rendered (Grid_Size / one frame's
    grid, one frame's grid the most common small dispatch), in us."""
    with (gzip.open(path, "rt") if path.endswith(".gz") else open(path)) as fp:
        rows = [r for r in csv.DictReader(fp) if kernel in r["Kernel_Name"] and "true" not in r["Kernel_Name"][:60]]
    if not rows:
        return None
    gkey = "Grid_Size" if "Grid_Size" in rows[0] else "Grid_Size_X"
    grids = [int(r[gkey]) for r in rows]
    g0 = min(grids)
    small = [g for g in grids if g < 1.5 * g0]
    one = max(set(small), key=small.count)
    # the union of the multi-frame launches' intervals (a chunk may run as
    # two concurrent launches on two streams, RT_MF_SPLIT) over their frames
    iv = []
    frames = 0
    for r, g in zip(rows, grids):
        f = int(round(g / one))
        if f > 1:
            iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
            frames += f
    dur, end = 0, None
    for a, b in sorted(iv):
        if end is None or a > end:
            dur += b - a
            end = b
        elif b > end:
            dur += b - end
            end = b
    return (dur / frames / 1e3, frames) if frames else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default="")
    ap.add_argument("--session", default="r04o", help="the bench session whose lines are checked")
    ap.add_argument("--trace-session", default="*", help="the session of the kernel traces and solo profiles (default: the latest by name)")
    a = ap.parse_args()
    pmc = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    rows = []
    for bp in sorted(glob.glob(os.path.join(a.dir, "bench", f"{a.session}_*.json"))):
        tag = os.path.splitext(os.path.basename(bp))[0]
        b = bench_line(bp)
        if not b or not b.get("roofline"):
            continue
        rf = b["roofline"]
        key = (rf.get("util_source") or "").split("[")[-1].split("]")[0] if rf.get("util_source") else None
        ent = pmc.get(key or "", {})
        # the solo-frame profile of the same arguments (`--inflight 1`: every
        # launch one frame, as bench.py's kernel time) when there is one
        # (bench/<session>_<config>.json pairs with rocprof/<session>_<config>_solo_*: any session, the latest)
        name = tag.split("_", 1)[1] if "_" in tag else tag
        if name.startswith("trace_") and name.endswith("_mf"):
            continue  # the profiled runs themselves (their traces are the reference)
        # repeats and variants of a configuration share its solo profile
        name = {"drv": "knot", "drv2": "knot", "drv_lanes": "knot", "knot_lanes": "knot", "trace_drv": "knot",
                "rehearse": "knot", "anim2": "anim", "anim3": "anim"}.get(name, name)
        st = sorted(glob.glob(os.path.join(a.dir, "rocprof", f"{a.trace_session}_{name}_solo_kernel_stats.csv")))[-1:]
        kern = "k_trace_flat" if rf.get("unit") == "TFLOP/s" else "k_trace_kd3"
        avg = stats_avg_us(st[0], "k_flat_chunk" if kern == "k_trace_flat" else kern) if st else None
        if key and key.endswith("_mf"):
            # multi-frame launches: the per-frame time of the launches in a
            # kernel trace of the bench's own command (no solo profile)
            tr = sorted(glob.glob(os.path.join(a.dir, "rocprof", f"{a.trace_session}_trace_{name}_mf_kernel_trace.csv*")))[-1:]
            pf = trace_per_frame_us(tr[0]) if tr else None
            avg = (pf[0], "multi-frame launches", pf[1]) if pf else None
        rec = None
        if avg and rf.get("unit") == "TFLOP/s" and rf.get("flops_per_launch"):
            # the flat kernel: the FLOP model's rate over the profiled kernel time
            rec = rf["flops_per_launch"] / (avg[0] * 1e-6) / 1e12 / rf["peak"]
        elif avg and ent.get("hbm_bytes_per_launch"):
            hbm = ent["hbm_bytes_per_launch"] / (avg[0] * 1e-6) / 1e9 / HBM
            rec = max(hbm, ent.get("valu_issue_util") or 0.0, ent.get("vmem_util") or 0.0)
        rows.append({"tag": tag, "workload": b.get("metric_workload") or b["config"].get("workload"),
                     "bench_frac": rf.get("frac"), "bound": rf.get("bound"), "bench_kernel_us": 1e3 * rf["kernel_ms_avg"],
                     "rocprof_avg_us": avg[0] if avg else None, "rocprof_calls": avg[2] if avg else None,
                     "rocprof_source": "per frame of multi-frame launches (kernel trace)" if key and key.endswith("_mf")
                     else "solo frames (--stats average)",
                     "pmc_key": key, "pmc_build": (ent.get("build_id") or "")[:16],
                     "vmem_util": ent.get("vmem_util"),
                     "traffic_over_compulsory": (round(ent["hbm_bytes_per_launch"] / rf["compulsory_bytes"], 3)
                                                 if ent.get("hbm_bytes_per_launch") and rf.get("compulsory_bytes") else None),
                     "bench_build": (b.get("build_id") or "")[:16], "recomputed_frac": rec,
                     "agree_5pct": (abs(rec - rf["frac"]) <= 0.05 * rf["frac"]) if rec and rf.get("frac") else None})
    out = ["| config | bound | bench frac | vmem_util | L2-miss bytes / compulsory | bench kernel us | rocprof us (calls or frames) | rocprof source | recomputed frac | within 5 % | PMC build = bench build |",
           "|---|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        out.append(f"| {r['tag']} ({r['workload']}) | {r['bound']} | {r['bench_frac']} | {r['vmem_util']} | "
                   f"{r['traffic_over_compulsory']} | {r['bench_kernel_us']:.2f} | "
                   f"{r['rocprof_avg_us'] and round(r['rocprof_avg_us'], 2)} ({r['rocprof_calls']}) | {r['rocprof_source']} | "
                   f"{r['recomputed_frac'] and round(r['recomputed_frac'], 4)} | {r['agree_5pct']} | "
                   f"{r['pmc_build'] == r['bench_build'] if r['pmc_build'] else 'no PMC entry'} |")
    text = "\n".join(out)
    print(text)
    if a.out:
        with open(a.out, "w") as fp:
            fp.write(text + "\n")
    return 0


if __name__ == "__main__":
    main()
