#!/usr/bin/env python3
"""Instruction mix of one kernel from rocprofv3 --pmc passes (VERDICT r04
item 3): per dispatch of the timed kernel instance, the median of each
counter over its dispatches of the dominant grid size (the timed frames'
launches; counting and warm-up renders have other instances), and the mix
per node visit with the visit counts of the bench line the passes ran.

    python tools/pmc_mix.py --kernel 'k_trace_kd3<16, false, false, false, 0>' \
        --bench gpurun_out/r05a/mix_knot_a.log gpurun_out/r05a/mix_knot_a gpurun_out/r05a/mix_knot_b

Counters are summed over the 8 XCDs by rocprofv3; SQ_INSTS_* count wave
instructions (one per wave64 instruction issued).
"""
import argparse
import csv
import glob
import gzip
import json
import os
import statistics
from collections import defaultdict


def rows(d):
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv*"), recursive=True):
        op = gzip.open if p.endswith(".gz") else open
        with op(p, "rt") as fp:
            yield from csv.DictReader(fp)


def bench_counts(log):
    for line in open(log):
        if line.startswith("{"):
            j = json.loads(line)
            return j["roofline"]["counts_per_launch"], j.get("build_id")
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", required=True, help="substring of the kernel name (the timed instance)")
    ap.add_argument("--bench", help="the bench log of one of the passes (its counts_per_launch)")
    ap.add_argument("--out")
    a = ap.parse_args()
    per = defaultdict(lambda: defaultdict(list))  # grid -> counter -> values per dispatch
    for d in a.dirs:
        disp = defaultdict(dict)
        for r in rows(d):
            if a.kernel not in r["Kernel_Name"]:
                continue
            disp[(r["Dispatch_Id"], r["Grid_Size"])][r["Counter_Name"]] = float(r["Counter_Value"])
        for (did, grid), cs in disp.items():
            for k, v in cs.items():
                per[grid][k].append(v)
    if not per:
        raise SystemExit("no dispatches of " + a.kernel)
    grid = max(per, key=lambda g: max(len(v) for v in per[g].values()))
    med = {k: statistics.median(v) for k, v in per[grid].items()}
    out = {"kernel": a.kernel, "grid_size": int(grid), "dispatches": max(len(v) for v in per[grid].values()),
           "per_dispatch": {k: round(v, 1) for k, v in sorted(med.items())}}
    if a.bench:
        cnt, bid = bench_counts(a.bench)
        out["bench_build_id"] = bid
        if cnt:
            visits = cnt["interior"] + cnt["leaf"]
            waves = med.get("SQ_WAVES")
            out["visits"] = {"interior": cnt["interior"], "leaf": cnt["leaf"], "total": visits}
            ratios = {}
            for k, v in med.items():
                if k.startswith("SQ_INSTS"):
                    ratios[k + "_per_visit"] = round(v / visits, 3)
                    if waves:
                        ratios[k + "_per_wave"] = round(v / waves, 1)
            out["ratios"] = ratios
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as fp:
            fp.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
