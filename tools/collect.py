#!/usr/bin/env python3
"""Copy a session's results from gpurun_out/<tag>/ into profiles/<round>/:
every bench JSON line -> bench/<tag>_<step>.json, every rocprofv3 --stats
summary -> rocprof/<tag>_<dir>_kernel_stats.csv (and a trace_* directory's
gzipped kernel trace beside it), every pmc_traffic_*.json ->
pmc/, tool JSON outputs (ranks_*, anim_*) -> ranks/ or anim/, and the GPU
test-suite tail -> pytest_gpu_<tag>.txt.

    python tools/collect.py r04l [--round r04]
"""
import argparse
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--round", default="r04")
    a = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", a.tag)
    dst = os.path.join(ROOT, "profiles", a.round)
    for sub in ("bench", "rocprof", "pmc", "ranks", "anim"):
        os.makedirs(os.path.join(dst, sub), exist_ok=True)
    n = 0
    for log in sorted(glob.glob(os.path.join(src, "*.log"))):
        step = os.path.splitext(os.path.basename(log))[0]
        with open(log, errors="replace") as fp:
            text = fp.read()
        lines = [ln for ln in text.splitlines() if ln.startswith('{"metric"')]
        if lines:
            with open(os.path.join(dst, "bench", f"{a.tag}_{step}.json"), "w") as fp:
                fp.write(lines[-1] + "\n")
            n += 1
        if step.startswith("pt") or step.startswith("pytest"):
            tail = [ln for ln in text.splitlines() if ln.strip()][-40:]
            with open(os.path.join(dst, f"pytest_gpu_{a.tag}_{step}.txt"), "w") as fp:
                fp.write("\n".join(tail) + "\n")
            n += 1
    for st in sorted(glob.glob(os.path.join(src, "*", "*kernel_stats.csv"))):
        d = os.path.basename(os.path.dirname(st))
        shutil.copy(st, os.path.join(dst, "rocprof", f"{a.tag}_{d}_kernel_stats.csv"))
        n += 1
    for kt in sorted(glob.glob(os.path.join(src, "trace_*", "*kernel_trace.csv.gz"))):
        d = os.path.basename(os.path.dirname(kt))
        shutil.copy(kt, os.path.join(dst, "rocprof", f"{a.tag}_{d}_kernel_trace.csv.gz"))
        n += 1
    for pj in sorted(glob.glob(os.path.join(src, "pmc_traffic_*.json"))):
        key = os.path.basename(pj)[len("pmc_traffic_"):-len(".json")]
        shutil.copy(pj, os.path.join(dst, "pmc", f"{key}_{a.tag}.json"))
        n += 1
    for tj in sorted(glob.glob(os.path.join(src, "*.json"))):
        b = os.path.basename(tj)
        if b.startswith("pmc_traffic_"):
            continue
        sub = "ranks" if b.startswith("ranks") else "anim"
        shutil.copy(tj, os.path.join(dst, sub, f"{a.tag}_{b}"))
        n += 1
    print(json.dumps({"tag": a.tag, "copied": n, "to": os.path.relpath(dst, ROOT)}))


if __name__ == "__main__":
    main()
