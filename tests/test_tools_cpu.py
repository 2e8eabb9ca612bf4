"""CPU tests of the measurement tools the roofline figures rest on:
tools/pmc_traffic.py's per-frame normalisation of multi-frame launches and
tools/roofline_check.py's per-frame time from a kernel trace (synthetic
rocprofv3 CSVs)."""
import csv
import gzip
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

KERNEL = "void rt::(anonymous namespace)::k_trace_kd3<16, false, false, false, 0>(rt::TraceParams)"
COUNT = "void rt::(anonymous namespace)::k_trace_kd3<16, false, false, true, 0>(rt::TraceParams)"
ONE = 4412 * 256  # one frame's grid (threads)


def _counter_csv(path, dispatches):
    """dispatches: (kernel name, grid size, {counter: value})."""
    cols = ["Correlation_Id", "Dispatch_Id", "Grid_Size", "Kernel_Name", "Counter_Name", "Counter_Value",
            "Start_Timestamp", "End_Timestamp"]
    with gzip.open(path, "wt") as fp:
        w = csv.DictWriter(fp, fieldnames=cols)
        w.writeheader()
        for i, (name, grid, ctrs) in enumerate(dispatches):
            for k, v in ctrs.items():
                w.writerow({"Correlation_Id": i, "Dispatch_Id": i, "Grid_Size": grid, "Kernel_Name": name,
                            "Counter_Name": k, "Counter_Value": v, "Start_Timestamp": 0, "End_Timestamp": 1})


@pytest.mark.parametrize("one_frame", [False, True])
def test_pmc_traffic_per_frame(tmp_path, one_frame):
    """Multi-frame dispatches (Grid_Size = k x one frame's grid) count k
    frames, single-frame dispatches are left out when multi-frame ones exist,
    and --one treats every dispatch as a frame."""
    d = tmp_path / "pass"
    d.mkdir()
    disp = [(COUNT, 2000 * 256, {"FETCH_SIZE": 999.0, "WRITE_SIZE": 999.0}),     # a counting frame: other kernel
            (KERNEL, ONE, {"FETCH_SIZE": 100.0, "WRITE_SIZE": 10.0}),            # one frame on its own
            (KERNEL, ONE, {"FETCH_SIZE": 100.0, "WRITE_SIZE": 10.0}),
            (KERNEL, 128 * ONE, {"FETCH_SIZE": 128 * 80.0, "WRITE_SIZE": 128 * 8.0}),   # 128 frames
            (KERNEL, 20 * ONE, {"FETCH_SIZE": 20 * 80.0, "WRITE_SIZE": 20 * 8.0})]      # 20 frames
    _counter_csv(str(d / "run_counter_collection.csv.gz"), disp)
    out = tmp_path / "t.json"
    args = [sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), "--out", str(out)]
    if one_frame:
        args.append("--one")
    subprocess.run(args + ["k", "k_trace_kd3<16, false, false, false", str(d)], check=True, capture_output=True)
    e = json.load(open(out))["k"]
    if one_frame:
        # every matching dispatch one frame: (100 + 100 + 10240 + 1600) / 4 KiB reads
        assert e["frames_per_dispatch"] == 1.0
        assert e["counters_per_frame"]["FETCH_SIZE"] == pytest.approx((200 + 128 * 80 + 20 * 80) / 4)
    else:
        # only the multi-frame launches, per frame: 80 KiB read, 8 KiB written
        assert e["frames_per_dispatch"] == pytest.approx(74.0)
        assert e["counters_per_frame"]["FETCH_SIZE"] == pytest.approx(80.0)
        assert e["hbm_bytes_per_frame"] == pytest.approx(2 * 80 * 1024 + 8 * 1024)
    assert e["build_id"]


def test_roofline_trace_per_frame(tmp_path):
    """The per-frame time of multi-frame launches in a kernel trace: their
    durations over their frames; single frames and other instances ignored."""
    import roofline_check as R
    p = tmp_path / "run_kernel_trace.csv.gz"
    rows = [(KERNEL, ONE, 0, 105_000), (KERNEL, ONE, 200_000, 305_000),
            (KERNEL, 128 * ONE, 400_000, 400_000 + 128 * 96_000), (KERNEL, 20 * ONE, 20_000_000, 20_000_000 + 20 * 97_000),
            (COUNT, 3000 * 256, 0, 1_000_000)]
    with gzip.open(p, "wt") as fp:
        w = csv.writer(fp)
        w.writerow(["Kernel_Name", "Grid_Size", "Start_Timestamp", "End_Timestamp"])
        for r in rows:
            w.writerow(r)
    us, frames = R.trace_per_frame_us(str(p))
    assert frames == 148
    assert us == pytest.approx((128 * 96 + 20 * 97) / 148)
