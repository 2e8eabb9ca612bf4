#!/usr/bin/env python3
"""One line per bench.py JSON result in the given logs / JSON files: FPS,
period, solo and in-flight kernel times, settle frames, loop kind, frame
check.

    python tools/bench_table.py gpurun_out/r04m/*.log
"""
import json
import os
import sys


def main():
    for f in sys.argv[1:]:
        try:
            lines = [x for x in open(f, errors="replace") if x.startswith('{"metric')]
        except OSError:
            continue
        if not lines:
            continue
        d = json.loads(lines[-1])
        r = d.get("roofline") or {}
        hst = d.get("host") or {}
        fc = d.get("frame_check") or {}
        print(f"{os.path.basename(f)[:24]:24s} {d.get('metric_workload', '')[:26]:26s} {d['value']:>10} "
              f"ms {d['ms_per_step']:.5f} solo {r.get('kernel_ms_avg')} timed {r.get('kernel_ms_avg_timed')} "
              f"settle {hst.get('settle_frames')} loop {hst.get('frames_in_flight')} g {hst.get('frame_group', '-')} "
              f"frac {r.get('frac')} fc {fc.get('matches_oracle', fc.get('gathered_equals_single_gpu_frame'))} "
              f"err {d.get('device_err')}")


if __name__ == "__main__":
    main()
