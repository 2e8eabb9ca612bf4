"""PLY input, CPU only.

The loader (csrc/scene_host.cpp rt_read_ply) parses ASCII bodies
line-parallel with std::from_chars, the same correctly rounded conversion as
strtof. Files whose records do not keep to one line take the token-by-token
reader instead (the reference's `>>` semantics, TD/read_ply.cpp:111-136).
It also reads binary_little_endian files, which the reference recognises but
does not read (TD/read_ply.cpp:28). Every result is compared with the
oracle's assembly of an independent parse.
"""
import os

import numpy as np
import pytest

from cpp_cuda_raytracer_dev_amd import _lib, raytracer as R, scenes
from oracle import _oracle as O


def test_binary_3_walls_matches_numpy_parse(tmp_path):
    """The reference's own binary mesh (Blender export: 8 float properties,
    uchar/uint face lists) against tests/golden/make_meshes.py's numpy parse."""
    z = np.load(os.path.join(scenes.MESH_DIR, "3_walls.npz"), allow_pickle=False)
    p = tmp_path / "3_walls.ply"
    p.write_bytes(z["ply_bytes"].tobytes())
    pts, n, leafs = R.read_ply(str(p), 0)
    opts, oleafs = O.assemble(z["verts"], z["arity"], z["idx"])
    assert n == 36 and pts.tobytes() == opts.tobytes()
    for f in ("x0", "x1", "y0", "y1", "z0", "z1"):
        assert leafs[f].tobytes() == oleafs[f].tobytes()


def _write_binary_ply(path, verts64, faces, extra_elem=True):
    """Binary little-endian PLY: double x/y/z between other properties, an
    unrelated element first, uchar/int face lists and a trailing face property."""
    nv, nf = len(verts64), len(faces)
    hdr = ["ply", "format binary_little_endian 1.0", "comment synthetic"]
    if extra_elem:
        hdr += ["element material 2", "property uchar r", "property float shininess"]
    hdr += [f"element vertex {nv}", "property ushort id", "property double x", "property double y",
            "property double z", "property float confidence",
            f"element face {nf}", "property list uchar int vertex_indices", "property short flags", "end_header"]
    out = bytearray(("\n".join(hdr) + "\n").encode())
    if extra_elem:
        out += np.array([(7, 0.5), (9, 0.25)], np.dtype([("r", "u1"), ("s", "<f4")])).tobytes()
    vdt = np.dtype([("id", "<u2"), ("x", "<f8"), ("y", "<f8"), ("z", "<f8"), ("c", "<f4")])
    rec = np.zeros(nv, vdt)
    rec["id"] = np.arange(nv) % 65536
    rec["x"], rec["y"], rec["z"] = verts64[:, 0], verts64[:, 1], verts64[:, 2]
    rec["c"] = 0.5
    out += rec.tobytes()
    for f in faces:
        out += np.array([len(f)], np.uint8).tobytes() + np.array(f, "<i4").tobytes() + np.array([3], "<i2").tobytes()
    path.write_bytes(bytes(out))


def _mesh(seed=5, nv=500, nf=700):
    rng = np.random.default_rng(seed)
    v64 = rng.normal(size=(nv, 3)) * 0.1
    faces = [[int(x) for x in rng.choice(nv, 3 if k % 3 else 4, replace=False)] for k in range(nf)]
    return v64, faces


def test_binary_synthetic_equals_ascii_and_oracle(tmp_path):
    v64, faces = _mesh()
    b = tmp_path / "m.ply"
    _write_binary_ply(b, v64, faces)
    pts, n, _ = R.read_ply(str(b), 0)
    v32 = v64.astype(np.float32)  # double coordinates round to float once
    a = np.array([len(f) for f in faces], np.int32)
    ix = np.array([i for f in faces for i in f], np.int32)
    opts, _ = O.assemble(v32, a, ix)
    assert n == len(opts) and pts.tobytes() == opts.tobytes()
    # the same mesh as ASCII (9 significant digits round-trip float32)
    t = tmp_path / "m_ascii.ply"
    lines = ["ply", "format ascii 1.0", f"element vertex {len(v32)}", "property float x", "property float y",
             "property float z", f"element face {len(faces)}", "property list uchar int vertex_indices",
             "end_header"]
    lines += [" ".join(f"{x:.9g}" for x in row) for row in v32]
    lines += [" ".join(str(x) for x in [len(f)] + f) for f in faces]
    t.write_text("\n".join(lines) + "\n")
    apts, an, _ = R.read_ply(str(t), 0)
    assert an == n and apts.tobytes() == pts.tobytes()
    assert apts.tobytes() == O.read_ply(str(t), 0)[0].tobytes()


@pytest.mark.parametrize("mode,per", [(1, 5), (2, 6)])
def test_ascii_extra_vertex_fields(tmp_path, mode, per):
    """Loader modes 1 and 2 (TD/WinMain.cpp:93-109): 5 or 6 numbers per vertex."""
    v64, faces = _mesh(seed=7, nv=300, nf=400)
    v32 = v64.astype(np.float32)
    t = tmp_path / "m.ply"
    lines = ["ply", "format ascii 1.0", f"element vertex {len(v32)}", f"element face {len(faces)}", "end_header"]
    lines += [" ".join(f"{x:.9g}" for x in list(row) + [0.25] * (per - 3)) for row in v32]
    lines += [" ".join(str(x) for x in [len(f)] + f) for f in faces]
    t.write_text("\n".join(lines) + "\n")
    pts, n, _ = R.read_ply(str(t), mode)
    assert pts.tobytes() == O.read_ply(str(t), mode)[0].tobytes()


def test_ascii_token_fallback(tmp_path):
    """Records split or joined across lines take the token reader and still
    equal the oracle's loader."""
    p = tmp_path / "odd.ply"
    p.write_text("ply\nformat ascii 1.0\nelement vertex 4\nelement face 2\nend_header\n"
                 "0 0 0 1 0 0\n0 1 0\n\n1 1 0.5\n3 0 1 2 3\n1 3 2\n")
    pts, n, _ = R.read_ply(str(p), 0)
    opts, _ = O.read_ply(str(p), 0)
    assert n == 2 and pts.tobytes() == opts.tobytes()


def test_binary_errors(tmp_path):
    p = tmp_path / "big.ply"
    p.write_bytes(b"ply\nformat binary_big_endian 1.0\nelement vertex 0\nelement face 0\nend_header\n")
    with pytest.raises(_lib.RtError):
        R.read_ply(str(p), 0)
    q = tmp_path / "trunc.ply"
    rng = np.random.default_rng(1)
    _write_binary_ply(q, rng.normal(size=(10, 3)), [[0, 1, 2]] * 5, extra_elem=False)
    q.write_bytes(q.read_bytes()[:-7])
    with pytest.raises(_lib.RtError):
        R.read_ply(str(q), 0)
