"""Regenerate tests/golden/meshes/*.npz from the reference's mesh files.

The reference's PLY files (data, not source) are stored as raw arrays:
verts [nv,3] float32 parsed with C strtof (the rounding of read_ply's
loader), arity [nf] int32 and idx (concatenated face indices).  Only
vertices' first three fields are kept (the loader discards the rest,
TD/read_ply.cpp:111-126).  Run in the container that has /root/reference.
"""
import ctypes
import os
import sys

import numpy as np

REF = "/root/reference/TEST_Dungeonrun"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "meshes")
MESHES = {"rabbit_70k": 5, "tester": 6, "dump": 5, "dump_test": 3}  # floats per vertex line

libc = ctypes.CDLL("libc.so.6")
libc.strtof.restype = ctypes.c_float
libc.strtof.argtypes = [ctypes.c_char_p, ctypes.c_void_p]


def parse(path, per_vertex):
    lines = open(path, "rb").read().split(b"\n")
    i = 0
    if lines[0].strip() == b"ply":
        i = 1
    if lines[i].strip().isdigit():
        nv, nf = int(lines[i]), int(lines[i + 1])
        i += 2
    else:
        nv = nf = None
        while lines[i].strip() != b"end_header":
            t = lines[i].split()
            if len(t) >= 3 and t[0] == b"element":
                if t[1] == b"vertex":
                    nv = int(t[2])
                if t[1] == b"face":
                    nf = int(t[2])
            i += 1
        i += 1
    toks = b" ".join(lines[i:]).split()
    vt = toks[: nv * per_vertex]
    verts = np.array([libc.strtof(t, None) for t in vt], np.float32).reshape(nv, per_vertex)[:, :3]
    rest = toks[nv * per_vertex:]
    arity, idx, k = [], [], 0
    for _ in range(nf):
        a = int(rest[k]); arity.append(a)
        idx.extend(int(x) for x in rest[k + 1: k + 1 + a]); k += 1 + a
    return np.ascontiguousarray(verts), np.array(arity, np.int32), np.array(idx, np.int32)


def main():
    os.makedirs(OUT, exist_ok=True)
    for name, per in MESHES.items():
        v, a, ix = parse(os.path.join(REF, name + ".ply"), per)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), verts=v, arity=a, idx=ix)
        print(name, v.shape, a.shape, ix.shape)
    return 0


if __name__ == "__main__":
    sys.exit(main())
