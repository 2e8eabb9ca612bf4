"""Summarise rocprofv3 --pmc passes of bench.py into profiles/pmc_traffic.json.

    python tools/pmc_traffic.py [--out file.json] [--one] <key> <kernel-substring> <pass_dir> [<pass_dir> ...]

Each pass directory holds one rocprofv3 --pmc run (counters collected in
separate passes: FETCH_SIZE and WRITE_SIZE do not fit one TCC pass).  The
matching kernel's counters are summed and divided by the frames the
dispatches rendered (a multi-frame launch renders many; see load()).  HBM bytes per launch
follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB, and on
gfx950 FETCH_SIZE reports half the bytes of 16-B-per-lane reads, so the read
side is doubled ("hbm_bytes_per_launch"); the raw sum is kept beside it.
"""
import csv
import glob
import gzip
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(pass_dir, kernel_sub, one_frame=False):
    """Per frame: every counter summed over the matching dispatches and
    divided by the frames they rendered.  A multi-frame launch
    (RT_LOOP_MULTIFRAME) renders Grid_Size / (one frame's grid) frames, one
    frame's grid being the most common of the small dispatches (the frames a
    run renders one at a time); when a run has multi-frame launches only
    those count (the mode bench.py times), else every dispatch is a frame."""
    rows = []
    paths = glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True)
    paths += glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv.gz"), recursive=True)  # session.sh
    for path in paths:
        with (gzip.open(path, "rt") if path.endswith(".gz") else open(path)) as fp:
            for row in csv.DictReader(fp):
                if kernel_sub in row.get("Kernel_Name", ""):
                    rows.append(row)
    if not rows:
        return {}, {}, 1.0
    grids = [int(r["Grid_Size"]) for r in rows if r.get("Grid_Size")]
    frames_of = lambda r: 1
    if grids and not one_frame:
        g0 = min(grids)
        small = [g for g in grids if g < 1.5 * g0]
        one = max(set(small), key=small.count)
        frames_of = lambda r: max(1, int(round(int(r["Grid_Size"]) / one)))
        if any(frames_of(r) > 1 for r in rows):
            rows = [r for r in rows if frames_of(r) > 1]
    vals, nfr, ndisp = defaultdict(float), defaultdict(int), defaultdict(int)
    for r in rows:
        vals[r["Counter_Name"]] += float(r["Counter_Value"])
        nfr[r["Counter_Name"]] += frames_of(r)
        ndisp[r["Counter_Name"]] += 1
    per_frame = {k: v / nfr[k] for k, v in vals.items() if nfr[k]}
    fpd = max(nfr[k] / ndisp[k] for k in ndisp) if ndisp else 1.0
    return per_frame, dict(ndisp), fpd


def main():
    argv = sys.argv[1:]
    out_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if argv and argv[0] == "--out":
        out_path, argv = argv[1], argv[2:]
    # --one: every dispatch is one frame (passes of --inflight 1 runs, whose
    # grids vary with a moving object's fine region)
    one_frame = bool(argv) and argv[0] == "--one"
    if one_frame:
        argv = argv[1:]
    key, kernel_sub, dirs = argv[0], argv[1], argv[2:]
    counters, n = {}, {}
    valu_util = None
    fpd = 1.0
    per_cu = {}  # busy / access counters per CU cycle of their own pass
    for d in dirs:
        c, m, f = load(d, kernel_sub, one_frame)
        fpd = max(fpd, f)
        if c.get("GRBM_GUI_ACTIVE"):
            # CU cycles of the pass: GRBM_GUI_ACTIVE is summed over the 8
            # XCDs (GRBM / 8 = the kernel's cycles), times the 256 CUs
            cu_cycles = c["GRBM_GUI_ACTIVE"] / 8.0 * 256.0
            for name in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum", "TD_TC_STALL_sum", "TCP_TOTAL_CACHE_ACCESSES_sum",
                         "TA_FLAT_READ_WAVEFRONTS_sum"):
                if name in c:
                    per_cu[name] = c[name] / cu_cycles
        if "SQ_INSTS_VALU" in c and c.get("GRBM_GUI_ACTIVE"):
            # VALU issue share of the chip's SIMD cycles in this pass: a wave64
            # VALU instruction issues over 2 cycles of a SIMD-32
            # (MI355X_MICROARCH.md), 1,024 SIMDs; the kernel's cycles are
            # GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs)
            valu_util = c["SQ_INSTS_VALU"] * 2.0 / (1024.0 * c["GRBM_GUI_ACTIVE"] / 8.0)
        c.pop("GRBM_GUI_ACTIVE", None)  # per pass; not merged
        counters.update(c)
        n.update(m)
    data = json.load(open(out_path)) if os.path.exists(out_path) else {}
    sys.path.insert(0, ROOT)
    from cpp_cuda_raytracer_dev_amd import build
    # the library the passes measured: this tree's (the binding refuses any
    # other), so bench.py can tell a stale entry from a current one
    entry = {"kernel": kernel_sub, "counters_per_frame": counters, "dispatches": n,
             "frames_per_dispatch": round(fpd, 2), "build_id": build.source_id()}
    if valu_util is not None:
        entry["valu_issue_util"] = round(valu_util, 4)
    if "TD_TD_BUSY_sum" in per_cu or "TA_TA_BUSY_sum" in per_cu:
        # the vector memory path per CU cycle (tools/ubench_l1.hip: a wave
        # load costs sum over its 16 lane quads of max(1, distinct 128-B
        # lines) TA / TD cycles, 16 at least for 64 lanes x 16 B; the data
        # unit also stalls on L1 misses): vmem_util is the data unit's busy
        # share, the busier of the two at every configuration measured
        entry["vmem"] = {k: round(v, 4) for k, v in per_cu.items()}
        entry["vmem_util"] = round(max(per_cu.get("TD_TD_BUSY_sum", 0.0), per_cu.get("TA_TA_BUSY_sum", 0.0)), 4)
    if "FETCH_SIZE" in counters and "WRITE_SIZE" in counters:
        fetch, write = counters["FETCH_SIZE"] * 1024.0, counters["WRITE_SIZE"] * 1024.0
        # per frame (one frame per launch unless multi-frame launches)
        entry["hbm_bytes_per_launch_raw"] = fetch + write
        entry["hbm_bytes_per_launch"] = 2.0 * fetch + write
        entry["hbm_bytes_per_frame"] = 2.0 * fetch + write
    if "TCC_HIT_sum" in counters and "TCC_MISS_sum" in counters:
        h, m = counters["TCC_HIT_sum"], counters["TCC_MISS_sum"]
        entry["l2_hit_rate"] = h / (h + m) if h + m else None
    c = counters
    if c.get("SQ_WAVE_CYCLES"):
        wc = c["SQ_WAVE_CYCLES"]
        # share of the waves' lifetime: waiting on anything, waiting for an
        # instruction's operands, issuing (any, VALU, LDS, scalar)
        entry["wave_time_split"] = {k: round(c[n] / wc, 4) for k, n in (
            ("wait_any", "SQ_WAIT_ANY"), ("wait_inst_any", "SQ_WAIT_INST_ANY"), ("active_any", "SQ_ACTIVE_INST_ANY"),
            ("active_valu", "SQ_ACTIVE_INST_VALU"), ("active_lds", "SQ_ACTIVE_INST_LDS"),
            ("wait_inst_lds", "SQ_WAIT_INST_LDS"), ("active_scalar", "SQ_ACTIVE_INST_SCA")) if n in c}
    if c.get("TCP_TCC_READ_REQ_sum"):
        entry["l1_miss_latency_cycles"] = c.get("TCP_TCC_READ_REQ_LATENCY_sum", 0.0) / c["TCP_TCC_READ_REQ_sum"]
        if c.get("TCP_TOTAL_CACHE_ACCESSES_sum"):
            entry["l1_miss_rate"] = c["TCP_TCC_READ_REQ_sum"] / c["TCP_TOTAL_CACHE_ACCESSES_sum"]
    if c.get("SQ_WAVES"):
        entry["per_wave"] = {k: round(c[n] / c["SQ_WAVES"], 2) for k, n in (
            ("valu_insts", "SQ_INSTS_VALU"), ("lds_insts", "SQ_INSTS_LDS"), ("salu_insts", "SQ_INSTS_SALU"),
            ("vmem_rd_insts", "SQ_INSTS_VMEM_RD"), ("branch_insts", "SQ_INSTS_BRANCH"),
            ("lds_bank_conflict_cycles", "SQ_LDS_BANK_CONFLICT")) if n in c}
    data[key] = entry
    json.dump(data, open(out_path, "w"), indent=1, sort_keys=True)
    print(json.dumps({key: entry}))


if __name__ == "__main__":
    main()
