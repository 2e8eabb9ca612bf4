#!/usr/bin/env python3
"""Vector memory path utilisation of the kd3 walk from rocprofv3 --pmc passes
(TA / TD / TCP counters; round 5, r05w / r05x).

    python tools/vmem_busy.py profiles/r05/pmc/vmem/r05w_knot_a_counter_collection.csv.gz [...]

Per pass: every k_trace_kd3 dispatch's counters summed, then divided by the
CU cycles of those dispatches.  GRBM_GUI_ACTIVE is summed over the 8 XCDs on
gfx950 (r05w: 8x the cycles the dispatches' frames take), so CU cycles =
GRBM_GUI_ACTIVE / 8 x 256 CUs.  A busy figure near 1 means that unit is busy
on every cycle of every CU.
"""
import collections
import csv
import gzip
import sys

N_XCD, N_CU = 8, 256


def summary(path):
    op = gzip.open if path.endswith(".gz") else open
    tot = collections.defaultdict(float)
    with op(path, "rt") as fp:
        for r in csv.DictReader(fp):
            if "k_trace_kd3" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    cu_cycles = tot.pop("GRBM_GUI_ACTIVE") / N_XCD * N_CU
    return {c: v / cu_cycles for c, v in sorted(tot.items())}


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(p)
        for c, v in summary(p).items():
            print(f"  {c:40s} {v:8.3f} per CU cycle")
