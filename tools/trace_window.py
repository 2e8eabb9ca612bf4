#!/usr/bin/env python3
"""The timed window of a short bench run from a rocprofv3 kernel + memory-copy
trace: the last N render launches (the timed frames of
`bench.py --steps N`), every kernel and copy between the first's start and the
last's end, each render's queue, start / end relative to the window, and where
the window's time goes (renders running, copies, nothing at all).

    python tools/trace_window.py <dir with *_kernel_trace.csv[.gz]> [--last 20] [--kernel k_trace_kd3]
"""
import argparse
import csv
import glob
import gzip
import os

import numpy as np


def rows(path):
    with (gzip.open(path, "rt") if path.endswith(".gz") else open(path)) as fp:
        return list(csv.DictReader(fp))


def find(d, what):
    for pat in (f"**/*{what}.csv", f"**/*{what}.csv.gz"):
        got = glob.glob(os.path.join(d, pat), recursive=True)
        if got:
            return got[0]
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=20)
    ap.add_argument("--kernel", default="k_trace_kd3")
    ap.add_argument("--chunks", type=int, default=0,
                    help="instead: every render launch of the trace in chunks of this many, mean duration and start")
    ap.add_argument("--skip", type=int, default=0,
                    help="renders after the window (bench --solo-when after: 20 + 5 x 200 solo frames follow it)")
    a = ap.parse_args()
    kt = rows(find(a.dir, "kernel_trace"))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:60],
           r.get("Queue_Id", r.get("Stream_Id", "?"))) for r in kt]
    mp = find(a.dir, "memory_copy_trace")
    if mp:
        for r in rows(mp):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       "C " + r.get("Direction", r.get("Operation", "copy")) + f" {r.get('Size', '?')} B", "dma"))
    ev.sort()
    rend = [e for e in ev if e[2].startswith("K") and a.kernel in e[2]]
    if a.chunks > 0:
        t00 = rend[0][0]
        print(f"{len(rend)} render launches; per chunk of {a.chunks}: first start (ms), mean / min duration (us)")
        for i in range(0, len(rend), a.chunks):
            d = [(e - s) / 1e3 for s, e, _, _ in rend[i:i + a.chunks]]
            print(f"  {i:6d} {(rend[i][0] - t00) / 1e6:9.2f} {np.mean(d):8.1f} {min(d):8.1f}")
        return
    rend = rend[len(rend) - a.last - a.skip:len(rend) - a.skip]
    t0, t1 = rend[0][0], rend[-1][1]
    win = [e for e in ev if e[1] >= t0 and e[0] <= t1]
    print(f"window: {a.last} renders, {(t1 - t0) / 1e3:.1f} us first start -> last end "
          f"({(t1 - t0) / 1e3 / a.last:.2f} us per frame)")
    for s, e, n, q in win:
        print(f"  {(s - t0) / 1e3:9.2f} {(e - t0) / 1e3:9.2f} {(e - s) / 1e3:8.2f}  q{q:>4}  {n}")
    # time with no render running, and what runs in it
    busy = np.zeros(int((t1 - t0) // 100) + 1, bool)  # 100 ns bins
    for s, e, n, q in rend:
        busy[(s - t0) // 100:(e - t0) // 100 + 1] = True
    idle = (~busy).sum() * 0.1
    print(f"no render running: {idle:.1f} us of {(t1 - t0) / 1e3:.1f}")
    # the previous launch before the window (its gap is the launch latency of the timed call)
    prev = [e for e in ev if e[1] < t0]
    if prev:
        p = prev[-1]
        print(f"last event before the window ends {(t0 - p[1]) / 1e3:.1f} us before it: {p[2]}")


if __name__ == "__main__":
    main()
