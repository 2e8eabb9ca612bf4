#!/usr/bin/env python3
"""Timeline gaps from a rocprofv3 --kernel-trace csv: per kernel name the
count and mean duration, and for the named render kernel the distribution of
start-to-start periods and of the idle gap between one render's end and the
next render's start (what the frame loop adds beyond the kernel).

    python tools/trace_gaps.py <run_kernel_trace.csv> [--kernel k_trace_kd3] [--skip 50]
"""
import argparse
import csv

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="k_trace_kd3")
    ap.add_argument("--skip", type=int, default=50)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    ks.sort()
    by = {}
    for s, e, n in ks:
        by.setdefault(n[:90], []).append(e - s)
    for n, d in sorted(by.items(), key=lambda x: -sum(x[1])):
        print(f"{len(d):6d} x {np.mean(d) / 1e3:9.2f} us  {n}")
    r = [(s, e) for s, e, n in ks if a.kernel in n][a.skip:]
    st = np.array([x[0] for x in r], np.int64)
    en = np.array([x[1] for x in r], np.int64)
    per = np.diff(st) / 1e3
    gap = (st[1:] - en[:-1]) / 1e3
    q = lambda v: [round(float(np.percentile(v, p)), 2) for p in (10, 50, 90, 99)]
    print(f"{a.kernel}: n={len(r)} dur mean {np.mean(en - st) / 1e3:.2f} us; period p10/50/90/99 {q(per)}; "
          f"end->next start gap {q(gap)}")
    # what ran inside the gaps (other kernels overlapping the idle window)
    other = [(s, e, n) for s, e, n in ks if a.kernel not in n and s >= st[0]]
    if other:
        os_ = np.array([x[0] for x in other])
        idx = np.searchsorted(en, os_) - 1
        lag = [(s - en[i]) / 1e3 for (s, e, n), i in zip(other, idx) if 0 <= i < len(en)]
        print(f"other kernels: start after preceding render end p10/50/90 {q(lag) if lag else None}")


if __name__ == "__main__":
    main()
