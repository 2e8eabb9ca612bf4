#!/usr/bin/env python3
"""Emit a tools/session.sh plan that collects every PMC pass of one
bench.py configuration (replaces round 2's pmc_*.sh scripts), then
summarises them into profiles/pmc_traffic.json with tools/pmc_traffic.py.

    python tools/pmc_plan.py [--own] <key> <kernel-substring> [bench args...] > plan
    tools/session.sh <tag> plan

One pass per counter group (rocprofv3 --pmc, counters only, no trace
domains), each within the gfx950 slot limits (SQ 8, TCC 4 with FETCH_SIZE
taking 3 and WRITE_SIZE 2, TCP 4, GRBM 2).  The bench runs one frame in
flight (--inflight 1) so every dispatch is a whole frame on its own, or with
--own its default loop (multi-frame launches where they apply: the passes
then count per frame, tools/pmc_traffic.py) without the solo pass.
"""
import shlex
import sys

PASSES = [
    ("fetch", "FETCH_SIZE GRBM_GUI_ACTIVE"),
    ("write", "WRITE_SIZE GRBM_GUI_ACTIVE"),
    ("tcc", "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"),
    ("sqwave", "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY "
               "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"),
    ("sqlds", "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS "
              "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"),
    ("tcp", "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"),
    # the vector memory path (round 6, verdict r05 item 4): address and data
    # units' busy cycles, the data unit's stalls on the L1, wave loads
    ("vmem", "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE"),
]


def main():
    if len(sys.argv) < 3 or (sys.argv[1] == "--own" and len(sys.argv) < 4):
        print(__doc__, file=sys.stderr)
        return 2
    argv = sys.argv[1:]
    own = argv[0] == "--own"  # the bench's own frame loop (multi-frame launches), without its solo pass
    if own:
        argv = argv[1:]
    key, ksub, args = argv[0], argv[1], argv[2:]
    bench = ("python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline "
             + ("--solo-frames 0 " if own else "--inflight 1 ") + " ".join(shlex.quote(a) for a in args))
    print(f"# PMC passes of [{key}] ({ksub}): bench.py {' '.join(args)}")
    for name, ctrs in PASSES:
        print(f"pmc_{key}_{name} 120 pmc pmc_{key}_{name} {ctrs} -- {bench}")
    print(f"pmc_{key}_summary 60 pmcsum {key} {shlex.quote(ksub)} " + " ".join(f"pmc_{key}_{n}" for n, _ in PASSES)
          + ("" if own else " --one"))
    return 0


if __name__ == "__main__":
    sys.exit(main())
