"""Scene inputs for the benchmark configs (BASELINE.json).

* ``fixture_mesh(name)``: the meshes that ship with the reference
  (rabbit_70k.ply, tester.ply, dump.ply, dump_test.ply), stored under
  tests/golden/meshes/ as raw vertex/face arrays (parsed with strtof, the
  rounding of the PLY loader).
* ``standin(name)``: seeded synthetic stand-ins for the two meshes missing
  from the reference (.MISSING_LARGE_BLOBS: dragon_vrip_mod.ply,
  happy_vrip_mod.ply).  Closed 2-manifold displaced blobs with exactly the
  public Stanford triangle counts and approximately their bounding boxes
  (SURVEY.md §8d).  Every report labels them "synthetic".
"""
from __future__ import annotations

import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MESH_DIR = os.path.join(ROOT, "tests", "golden", "meshes")

#: loader mode of each reference mesh (TD/WinMain.cpp:93-109)
FIXTURE_MODES = {"rabbit_70k": 1, "tester": 2, "dump": 1, "dump_test": 0}

STANDINS = {
    # name: (triangles, bbox lo, bbox hi, (U, V) main blob, (U, V) small blob)
    "dragon": (871_414, (-0.112, 0.052, -0.067), (0.093, 0.199, 0.054), (640, 681), (39, 14)),
    "happy": (1_087_716, (-0.047, 0.055, -0.037), (0.044, 0.248, 0.047), (720, 756), (43, 7)),
    # not a reference mesh: > 2^21 triangles, so its median tree is 22 levels
    # tall (kernel 3's former path-code limit was 21); dragon-sized box
    "big": (3_146_328, (-0.112, 0.052, -0.067), (0.093, 0.199, 0.054), (1536, 1025), (60, 6)),
    # not a reference mesh: the dragon's triangle count and box as a
    # noise-displaced (5, 12) torus-knot tube (SURVEY.md §8d's suggestion):
    # strands in front of strands, so a covered ray crosses ~1.9x the boxes
    # of the convex-ish blob (183 vs 98 interior visits per hit pixel at
    # 480x270).  (U, V) = curve samples x tube samples, then the small blob
    "knot": (871_414, (-0.112, 0.052, -0.067), (0.093, 0.199, 0.054), (3000, 145), (101, 8)),
}
STANDIN_SEED = 20221015

#: WinMain's camera (TD/WinMain.cpp:69-74): every view keeps its film and
#: focal length; only the position and look-at point change.
DEFAULT_VIEW = {"pos": (0.0, 0.1, -1.0), "look_at": (0.0, 0.1, 0.0)}
#: "fill" views put the object over >= 90 % of the pixels (README.md:19 quotes
#: "25 FPS at 90%+ pixel coverage" beside the default view's ~100 FPS): the
#: camera looks along +z at the object's box centre from closer in.  Found by
#: rendering the oracle at 192x108; the coverage at each resolution is
#: recorded with the frame hashes (tests/golden/frame_hashes.json).
FILL_VIEWS = {
    "dragon": {"pos": (-0.0097, 0.1309, -0.2312), "look_at": (-0.0097, 0.1309, -0.0061)},   # ~94 %
    "rabbit_70k": {"pos": (-0.0068, 0.0902, -0.1419), "look_at": (-0.0068, 0.0902, -0.0015)},  # ~95 %
    "happy": {"pos": (-0.0037, 0.1512, -0.1147), "look_at": (-0.0037, 0.1512, 0.0061)},
}


def view(scene: str, name: str = "default") -> dict:
    """Camera position / look-at of a named view ("default" or "fill")."""
    if name == "default":
        return dict(DEFAULT_VIEW)
    if name == "fill":
        return dict(FILL_VIEWS[scene])
    raise KeyError(f"unknown view {name!r} (default, fill)")


def fixture_mesh(name: str):
    """(verts [nv,3] f32, arity [nf] i32, idx [sum arity] i32) of a reference mesh."""
    z = np.load(os.path.join(MESH_DIR, f"{name}.npz"), allow_pickle=False)
    return z["verts"], z["arity"], z["idx"]


def _uv_sphere(U: int, V: int):
    """Unit-sphere vertices and triangle faces with 2*U*(V-1) triangles:
    two poles, V-1 rings of U vertices."""
    theta = np.pi * (np.arange(1, V, dtype=np.float64) / V)            # ring latitudes
    phi = 2 * np.pi * (np.arange(U, dtype=np.float64) / U)
    st, ct = np.sin(theta)[:, None], np.cos(theta)[:, None]
    ring = np.stack([st * np.cos(phi)[None, :], ct * np.ones((1, U)), st * np.sin(phi)[None, :]], -1)
    verts = np.concatenate([[[0.0, 1.0, 0.0]], ring.reshape(-1, 3), [[0.0, -1.0, 0.0]]])
    south = 1 + (V - 1) * U
    j = np.arange(U)
    jn = (j + 1) % U
    faces = [np.stack([np.zeros(U, np.int64), 1 + jn, 1 + j], -1)]
    for r in range(V - 2):
        a, b = 1 + r * U + j, 1 + r * U + jn
        c, d = a + U, b + U
        faces.append(np.stack([a, b, d], -1))
        faces.append(np.stack([a, d, c], -1))
    last = 1 + (V - 2) * U
    faces.append(np.stack([last + j, last + jn, np.full(U, south)], -1))
    return verts, np.concatenate(faces).astype(np.int32)


def _noise(v: np.ndarray, rng: np.random.Generator, octaves: int, amp: float) -> np.ndarray:
    """1 + a sum of seeded plane waves at the points v (a radial factor)."""
    r = np.ones(len(v))
    for o in range(octaves):
        k = 3.0 * (1.9 ** o)
        for _ in range(4):
            d = rng.normal(size=3)
            d /= np.linalg.norm(d)
            ph = rng.uniform(0, 2 * np.pi)
            r += (amp / (1.7 ** o)) * np.sin(k * (v @ d) + ph)
    return r


def _displace(v: np.ndarray, rng: np.random.Generator, octaves: int, amp: float) -> np.ndarray:
    return v * _noise(v, rng, octaves, amp)[:, None]


def _knot_tube(U: int, V: int, rng: np.random.Generator, p: int = 5, q: int = 12, tube: float = 0.28):
    """A closed tube around the (p, q) torus knot: U rings of V vertices
    (2*U*V triangles, torus topology), parallel-transported frames with the
    closing twist spread along the curve, and a noise-displaced radius."""
    t = 2 * np.pi * np.arange(U, dtype=np.float64) / U
    r = 2.0 + np.cos(q * t)
    curve = np.stack([r * np.cos(p * t), r * np.sin(p * t), 1.1 * np.sin(q * t)], -1)
    tan = np.roll(curve, -1, 0) - np.roll(curve, 1, 0)
    tan /= np.linalg.norm(tan, axis=1, keepdims=True)
    nrm = np.zeros_like(curve)
    n = np.cross(tan[0], [0.0, 0.0, 1.0])
    n /= np.linalg.norm(n)
    for i in range(U):  # parallel transport: remove the tangential part
        n = n - tan[i] * (n @ tan[i])
        n /= np.linalg.norm(n)
        nrm[i] = n
    bin_ = np.cross(tan, nrm)
    # the transported frame comes back rotated by `twist`: spread it out
    n_end = nrm[-1] - tan[0] * (nrm[-1] @ tan[0])
    twist = np.arctan2(n_end @ bin_[0], n_end @ nrm[0])
    a = -twist * np.arange(U) / U
    nrm, bin_ = (np.cos(a)[:, None] * nrm + np.sin(a)[:, None] * bin_,
                 -np.sin(a)[:, None] * nrm + np.cos(a)[:, None] * bin_)
    th = 2 * np.pi * np.arange(V, dtype=np.float64) / V
    ring = np.cos(th)[None, :, None] * nrm[:, None, :] + np.sin(th)[None, :, None] * bin_[:, None, :]
    base = curve[:, None, :] + tube * ring
    rad = _noise(base.reshape(-1, 3) / 3.0, rng, octaves=6, amp=0.05).reshape(U, V, 1)
    verts = curve[:, None, :] + tube * ring * rad
    i = np.arange(U)[:, None]
    j = np.arange(V)[None, :]
    a0 = i * V + j
    b0 = i * V + (j + 1) % V
    c0 = ((i + 1) % U) * V + j
    d0 = ((i + 1) % U) * V + (j + 1) % V
    faces = np.concatenate([np.stack([a0, b0, d0], -1).reshape(-1, 3), np.stack([a0, d0, c0], -1).reshape(-1, 3)])
    return verts.reshape(-1, 3), faces.astype(np.int32)


def standin(name: str):
    """Synthetic stand-in mesh: (verts [nv,3] f32, faces [nf,3] i32)."""
    ntri, lo, hi, (U, V), (u2, v2) = STANDINS[name]
    rng = np.random.default_rng(STANDIN_SEED + {"dragon": 0, "happy": 1, "big": 2, "knot": 3}[name])
    lo, hi = np.asarray(lo), np.asarray(hi)
    c, half = (lo + hi) / 2, (hi - lo) / 2
    if name == "knot":
        v, f = _knot_tube(U, V, rng)
        v = v - (v.max(axis=0) + v.min(axis=0)) / 2
    else:
        v, f = _uv_sphere(U, V)
        v = _displace(v, rng, octaves=6, amp=0.06)
    v = v / np.abs(v).max(axis=0)  # fill the box
    body = c + half * v
    # a small closed blob near the +x end (head/eye), fully inside the box
    v2, f2 = _uv_sphere(u2, v2)
    eye = c + half * np.array([0.78, 0.45, 0.30]) + 0.06 * half.min() * v2
    verts = np.concatenate([body, eye]).astype(np.float32)
    faces = np.concatenate([f, f2 + len(body)]).astype(np.int32)
    assert len(faces) == ntri, (name, len(faces))
    return verts, faces


def mesh_arrays(name: str):
    """(verts [nv,3] f32, arity [nf] i32, idx i32) of a reference fixture or a
    stand-in, the input of read_ply's face assembly."""
    if name in STANDINS:
        v, f = standin(name)
        return v, np.full(len(f), 3, np.int32), np.ascontiguousarray(f, np.int32).reshape(-1)
    return fixture_mesh(name)


def faces_of(arity: np.ndarray, idx: np.ndarray):
    """Faces for raytracer.assemble_mesh: an [nf, k] array when every face has
    k vertices, else a list of per-face index lists."""
    if len(arity) and arity.min() == arity.max():
        return np.asarray(idx, np.int32).reshape(len(arity), -1)
    starts = np.r_[0, np.cumsum(arity)[:-1]]
    return [list(idx[s:s + k]) for s, k in zip(starts, arity)]


def mesh_sha(name: str) -> str:
    """SHA-256 of a mesh's vertex and face arrays: frame hashes recorded for a
    stand-in hold only where its (numpy-generated) vertices are the same."""
    import hashlib
    v, a, ix = mesh_arrays(name)
    h = hashlib.sha256()
    for arr in (np.ascontiguousarray(v, np.float32), np.ascontiguousarray(a, np.int32),
                np.ascontiguousarray(ix, np.int32)):
        h.update(arr.tobytes())
    return h.hexdigest()


def write_ply(path: str, verts: np.ndarray, faces: np.ndarray) -> None:
    """Mode-0 ASCII PLY (x y z per vertex); %.9g round-trips float32."""
    with open(path, "w") as fp:
        fp.write(f"ply\nformat ascii 1.0\nelement vertex {len(verts)}\nproperty float x\nproperty float y\n"
                 f"property float z\nelement face {len(faces)}\nproperty list uchar int vertex_indices\n"
                 "end_header\n")
        np.savetxt(fp, verts.astype(np.float64), fmt="%.9g")
        arity = np.full((len(faces), 1), faces.shape[1], np.int64)
        np.savetxt(fp, np.concatenate([arity, faces.astype(np.int64)], 1), fmt="%d")
