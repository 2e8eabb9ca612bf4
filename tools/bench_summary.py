#!/usr/bin/env python3
"""Summarise bench.py JSON lines from log files: one row per line."""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        line = line.strip()
        if not line.startswith("{"):
            continue
        try:
            r = json.loads(line)
        except ValueError:
            continue
        if not isinstance(r, dict) or "value" not in r:  # another tool's JSON (pmc_traffic.py)
            continue
        rf = r.get("roofline") or {}
        cb = r.get("cpu_baseline") or {}
        fc = r.get("frame_check") or {}
        print(f"{path.split('/')[-1][:28]:28s} {r['value']:>10} {r['unit']:9s} ms {r['ms_per_step']:<8} "
              f"cov {r['config'].get('coverage')} kern_ms {rf.get('kernel_ms_avg')} {rf.get('unit')} "
              f"ach {rf.get('achieved')} frac {rf.get('frac')} err {r.get('device_err')} "
              f"fc {fc.get('matches_oracle', fc.get('gathered_equals_single_gpu_frame'))} "
              f"cpu {cb.get('value')}/{cb.get('value_1thread')} ({cb.get('cores')}t)")
