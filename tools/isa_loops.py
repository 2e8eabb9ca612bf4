#!/usr/bin/env python3
"""Static instruction mix of a kernel's loops from hipcc's device assembly.

    hipcc <library flags> --offload-device-only -S -o kd.s csrc/rt_kd_dispatch.hip -DRT_KD_T=0 ...
    python tools/isa_loops.py kd.s --kernel 'k_trace_kd3ILi16ELb0ELb0ELb0ELi0E' [--blocks]

Groups the kernel's basic blocks by the innermost loop header LLVM names in
its block comments ("in Loop: Header=BBx_y Depth=d"), and prints, per loop,
the instruction count by class: VALU (v_*), of which f64 and transcendental,
SALU (s_* but branches, waits and barriers), LDS (ds_*), VMEM (global_* /
buffer_* / flat_*), SMEM (s_load / s_buffer_load), branches and waits.  A
loop's count is the sum over its blocks (every path of a branchy body once),
so it is an upper bound of one iteration's issue when the body diverges; with
--blocks each block is listed too.  Used to compare builds of the traversal
loop without a GPU (round 5).
"""
import argparse
import re
import sys
from collections import OrderedDict, defaultdict

CLASSES = ("valu", "v_f64", "v_trans", "v_cmp", "v_cndmask", "salu", "lds", "vmem", "smem", "branch", "wait", "other")
TRANS = re.compile(r"^v_(rcp|rsq|sqrt|exp|log|sin|cos|div_scale|div_fmas|div_fixup|frexp|ldexp)")


def classify(op: str) -> list:
    if op.startswith("v_"):
        out = ["valu"]
        if "_f64" in op:
            out.append("v_f64")
        if TRANS.match(op):
            out.append("v_trans")
        if op.startswith("v_cmp") or op.startswith("v_cmpx"):
            out.append("v_cmp")
        if op.startswith("v_cndmask"):
            out.append("v_cndmask")
        return out
    if op.startswith("ds_"):
        return ["lds"]
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return ["vmem"]
    if op.startswith(("s_load", "s_buffer_load")):
        return ["smem"]
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc")):
        return ["branch"]
    if op.startswith(("s_waitcnt", "s_barrier", "s_nop", "s_sleep", "s_endpgm")):
        return ["wait"]
    if op.startswith("s_"):
        return ["salu"]
    return ["other"]


def kernel_lines(path: str, pat: str):
    lines = open(path).read().splitlines()
    start = None
    for i, line in enumerate(lines):
        if start is None and re.match(r"^_Z\S*" + pat + r"\S*:", line):
            start = i
        elif start is not None and line.startswith(".Lfunc_end"):
            return lines[start:i]
    if start is None:
        sys.exit(f"no kernel matching {pat!r} in {path}")
    return lines[start:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--kernel", required=True, help="regex on the mangled kernel name")
    ap.add_argument("--blocks", action="store_true")
    ap.add_argument("--min", type=int, default=20, help="loops with fewer instructions are not printed")
    a = ap.parse_args()
    blocks = OrderedDict()  # label -> (header or None, depth, counts)
    cur = None
    total = defaultdict(int)
    for line in kernel_lines(a.asm, a.kernel):
        m = re.match(r"^(\.LBB\w+|; %bb\.\d+):?\s*(.*)$", line)
        if m:
            label = m.group(1).replace("; %", "")
            hdr = re.search(r"Header=(BB\w+) Depth=(\d+)", m.group(2))
            own = re.search(r"Loop Header: Depth=(\d+)", m.group(2))
            if own:
                header, depth = label.lstrip(".L"), int(own.group(1))
            elif hdr:
                header, depth = hdr.group(1), int(hdr.group(2))
            else:
                header, depth = None, 0
            cur = label
            blocks[cur] = (header, depth, defaultdict(int))
            continue
        s = line.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op = s.split()[0]
        if cur is None:
            cur = "entry"
            blocks[cur] = (None, 0, defaultdict(int))
        for c in classify(op):
            blocks[cur][2][c] += 1
            total[c] += 1
    loops = OrderedDict()
    for label, (hdr, depth, cnt) in blocks.items():
        key = hdr or "(no loop)"
        ent = loops.setdefault(key, [depth, defaultdict(int), []])
        ent[0] = max(ent[0], depth)
        for c, v in cnt.items():
            ent[1][c] += v
        ent[2].append((label, cnt))
    hdrs = "".join(f"{c:>9}" for c in CLASSES)
    print(f"{'loop header':<16}{'depth':>6}{'blocks':>7}{hdrs}")
    for key, (depth, cnt, bl) in loops.items():
        if sum(cnt[c] for c in ("valu", "salu", "lds", "vmem", "smem", "branch", "wait", "other")) < a.min:
            continue
        print(f"{key:<16}{depth:>6}{len(bl):>7}" + "".join(f"{cnt[c]:>9}" for c in CLASSES))
        if a.blocks:
            for label, c in bl:
                print(f"    {label:<20}" + "".join(f"{c[k]:>9}" for k in CLASSES))
    print(f"{'kernel':<16}{'':>6}{len(blocks):>7}" + "".join(f"{total[c]:>9}" for c in CLASSES))


if __name__ == "__main__":
    main()
