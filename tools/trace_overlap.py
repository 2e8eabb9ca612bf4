#!/usr/bin/env python3
"""Frames-in-flight timeline from a rocprofv3 --kernel-trace csv: over the
last N render launches, the render period (start to start of consecutive
frames, any lane), each render's duration, and the time the GPU runs no
render at all (gaps in the union of render intervals).

    python tools/trace_overlap.py <run_kernel_trace.csv> [--kernel k_trace_kd3] [--last 500]
"""
import argparse
import csv

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="k_trace_kd3")
    ap.add_argument("--last", type=int, default=500)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace))]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    rend = [(s, e) for s, e, n in ks if a.kernel in n][-a.last:]
    t0, t1 = rend[0][0], rend[-1][1]
    dur = np.array([e - s for s, e in rend]) / 1e3
    # union of render intervals
    busy, cur_s, cur_e = 0, None, None
    for s, e in rend:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = (t1 - t0) / 1e3
    others = [(s, e, n) for s, e, n in ks if a.kernel not in n and t0 <= s <= t1]
    kinds = {}
    for s, e, n in others:
        k = n.split("(")[0][-40:]
        kinds.setdefault(k, []).append((e - s) / 1e3)
    print(f"renders {len(rend)}: period {span / len(rend):.2f} us, duration mean {dur.mean():.2f} us "
          f"(p10 {np.percentile(dur, 10):.1f}, p90 {np.percentile(dur, 90):.1f}), "
          f"no render running {100 * (1 - busy / 1e3 / span):.1f} % of the span")
    for k, v in kinds.items():
        print(f"  other: {len(v)} x {np.mean(v):.2f} us  {k}")


if __name__ == "__main__":
    main()
