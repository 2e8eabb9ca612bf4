"""Regenerate tests/golden/meshes/*.npz from the reference's mesh files.

3_walls.ply is binary_little_endian (Blender export, 8 float properties per
vertex, uchar/uint face lists); the reference recognises the format but
reads no binary data (TD/read_ply.cpp:28).  It is parsed here with numpy
alone and stored with its raw bytes, so the C loader's binary path can be
checked against an independent parse.

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


_NP = {"char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "<i2", "int16": "<i2",
       "ushort": "<u2", "uint16": "<u2", "int": "<i4", "int32": "<i4", "uint": "<u4", "uint32": "<u4",
       "float": "<f4", "float32": "<f4", "double": "<f8", "float64": "<f8"}


def parse_binary(path):
    raw = open(path, "rb").read()
    end = raw.index(b"end_header\n") + len(b"end_header\n")
    elems = []
    for ln in raw[:end].decode().splitlines():
        t = ln.split()
        if t and t[0] == "element":
            elems.append((t[1], int(t[2]), []))
        elif t and t[0] == "property":
            elems[-1][2].append(("list", t[2], t[3], t[4]) if t[1] == "list" else (t[1], t[2]))
    off, verts, arity, idx = end, None, [], []
    for name, count, props in elems:
        if all(len(p) == 2 for p in props):
            dt = np.dtype([(p[1], _NP[p[0]]) for p in props])
            rec = np.frombuffer(raw, dt, count, off)
            off += count * dt.itemsize
            if name == "vertex":
                verts = np.stack([rec["x"], rec["y"], rec["z"]], 1).astype(np.float32)
            continue
        for _ in range(count):  # face element: one list property
            (_, ct, it, _) = props[0]
            n = int(np.frombuffer(raw, _NP[ct], 1, off)[0]); off += np.dtype(_NP[ct]).itemsize
            v = np.frombuffer(raw, _NP[it], n, off); off += n * np.dtype(_NP[it]).itemsize
            if name == "face":
                arity.append(n); idx.extend(int(x) for x in v)
    return raw, np.ascontiguousarray(verts), np.array(arity, np.int32), np.array(idx, np.int32)


def main():
    os.makedirs(OUT, exist_ok=True)
    raw, v, a, ix = parse_binary(os.path.join(REF, "3_walls.ply"))
    np.savez_compressed(os.path.join(OUT, "3_walls.npz"), verts=v, arity=a, idx=ix,
                        ply_bytes=np.frombuffer(raw, np.uint8))
    print("3_walls", v.shape, a.shape, ix.shape, len(raw), "bytes")
    for name, per in MESHES.items():
        v, a, ix = parse(os.path.join(REF, name + ".ply"), per)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), verts=v, arity=a, idx=ix)
        print(name, v.shape, a.shape, ix.shape)
    return 0


if __name__ == "__main__":
    sys.exit(main())
