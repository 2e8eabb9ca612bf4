"""Independent numpy restatement of the reference hot path (small scenes only).

TEST INFRASTRUCTURE ONLY.  Written separately from oracle/oracle.c to
cross-check it: float32 numpy arithmetic in the reference's evaluation
order, float64 exactly where the reference promotes (1e-16 epsilons,
`.6*`, `*.3`, `1.0/f`), pure-Python loops over rays and tree nodes.  Used by
tests/golden/make_golden.py to produce the committed fixtures and by
tests/test_oracle_crosscheck.py.  TD/ = TEST_Dungeonrun/ in the reference.
"""
from __future__ import annotations

import numpy as np

F = np.float32
D = np.float64
EPS = D(1e-16)                 # TD/vector.cuh:10-11
BG = 0x00F08200                # TD/Camera.cpp:72
IDENT = np.array([1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0], F)


def _bits(x):
    return int(np.array([x], F).view(np.uint32)[0])


def _from_bits(i):
    return np.array([i & 0xFFFFFFFF], np.uint32).view(F)[0]


def rsqrt(s, steps):
    """vector_norm (TD/vector.cpp:13-26, 8 steps) / device_inverse_sqrt (TD/vector.cuh:79-95, 21 steps)."""
    s = F(s)
    half = F(F(0.5) * s)
    y = _from_bits(0x5F375A86 - (_bits(half) >> 1))
    for _ in range(steps):
        y = F(y * F(F(1.5) - F(F(half * y) * y)))
    return y


def dev_normalize(x, y, z):
    s = F(F(F(x * x) + F(y * y)) + F(z * z))
    r = rsqrt(s, 21)
    return F(x * r), F(y * r), F(z * r)


def cross(a, b):
    return (F(F(a[1] * b[2]) - F(a[2] * b[1])), F(F(a[2] * b[0]) - F(a[0] * b[2])), F(F(a[0] * b[1]) - F(a[1] * b[0])))


def dot(a, b):
    return F(F(F(a[0] * b[0]) + F(a[1] * b[1])) + F(a[2] * b[2]))


# --------------------------------------------------------------- camera (a1, a2)

def camera(w, h, f_w=None, f_h=F(0.024), focal=F(0.055), pos=(0.0, 0.1, -1.0), la=(0.0, 0.1, 0.0),
           up=(0.0, 1.0, 0.0)):
    if f_w is None:
        f_w = F(F(F(w) / F(h)) * F(0.024))            # TD/WinMain.cpp:29,70
    pos = [F(v) for v in pos]; la = [F(v) for v in la]; up = [F(v) for v in up]
    pix_w, pix_h = F(F(f_w) / F(w)), F(F(f_h) / F(h))

    def norm4(v):
        s = F(F(F(v[0] * v[0]) + F(v[1] * v[1])) + F(v[2] * v[2]))
        s = rsqrt(s, 8)
        return [F(v[0] * s), F(v[1] * s), F(v[2] * s)]

    n = norm4([F(la[k] - pos[k]) for k in range(3)])
    tu = norm4(up)
    tu = list(cross(tu, n))
    nn = list(cross(n, tu))
    v = norm4(nn)
    v_mod = [F(c * pix_h) for c in v]
    n2 = norm4([F(la[k] - pos[k]) for k in range(3)])
    u = list(cross(v, n2))
    u_mod = [F(c * pix_w) for c in u]
    ay = F(h >> 1); ax = F(w >> 1)
    if not (h & 1): ay = F(D(ay) - 0.5)
    if not (w & 1): ax = F(D(ax) - 0.5)
    n_mod = [F(F(F(n[k] * F(focal)) - F(v_mod[k] * ay)) - F(u_mod[k] * ax)) for k in range(3)]
    return dict(w=w, h=h, pos=pos, n=n, u=u, v=v, n_mod=n_mod, u_mod=u_mod, v_mod=v_mod)


def primary_ray(cam, ix, iy):
    fx, fy = F(ix), F(iy)
    c = [F(F(cam["n_mod"][k] + F(cam["u_mod"][k] * fx)) + F(cam["v_mod"][k] * fy)) for k in range(3)]
    return dev_normalize(*c)


# ----------------------------------------------------------- mesh + KD (a11)

def assemble(verts, arity, idx):
    """TD/read_ply.cpp:67-149."""
    mn = lambda a, b: a if a < b else b  # noqa: E731
    mx = lambda a, b: a if a > b else b  # noqa: E731
    pts, boxes = [], []
    k = 0
    for a in arity:
        ids = list(idx[k:k + a]); k += a
        P = [verts[i] for i in ids]
        tris = [((P[0], P[1], P[2]), (P[0], P[1], P[2])), ((P[0], P[2], P[3]), (P[0], P[3], P[2]))] if a == 4 \
            else [((P[2], P[0], P[1]), (P[0], P[1], P[2]))]
        for stored, bx in tris:
            pts.append(np.concatenate(stored).astype(F))
            boxes.append([mn(bx[0][c], mn(bx[1][c], bx[2][c])) for c in range(3)] +
                         [mx(bx[0][c], mx(bx[1][c], bx[2][c])) for c in range(3)])
    return np.array(pts, F).reshape(-1, 9), np.array(boxes, F)   # boxes: x0 y0 z0 x1 y1 z1


def build_kd(boxes):
    """set_sorted_voxels + create_kd (TD/Trixel.h:135-473), via a literal merge sort."""
    n = len(boxes)
    # list k (cut order 0 x1,1 y1,2 z1,3 x0,4 y0,5 z0) -> column of boxes
    col = {0: 3, 1: 4, 2: 5, 3: 0, 4: 1, 5: 2}

    def msort(ids, c):                     # TD/sort.h:11-60, right run wins ties
        if len(ids) <= 1:
            return ids
        m = (len(ids) - 1) // 2 + 1
        L, R = msort(ids[:m], c), msort(ids[m:], c)
        out, i, j = [], 0, 0
        while i < len(L) and j < len(R):
            if boxes[L[i], c] < boxes[R[j], c]:
                out.append(L[i]); i += 1
            else:
                out.append(R[j]); j += 1
        return out + L[i:] + R[j:]

    lists = [msort(list(range(n)), col[k]) for k in range(6)]
    key = lambda k, p: boxes[lists[k][p], col[k]]  # noqa: E731
    nodes = [dict(l=0, m=(n - 1) // 2, r=n - 1, parent=0, cut=5)]
    nodes[0].update(x0=key(3, 0), x1=key(0, n - 1), y0=key(4, 0), y1=key(1, n - 1), z0=key(5, 0), z1=key(2, n - 1))
    rd = 0
    while rd < len(nodes):
        nd = nodes[rd]
        l, m, r = nd["l"], nd["m"], nd["r"]
        best, cut = F(key(0, r) - key(0, l)), 0
        for k in (3, 1, 4, 2, 5):
            span = F(key(k, r) - key(k, l))
            if span > best:
                best, cut = span, k
        if r == l:
            nd.update(leaf=1, tri=lists[0][l], cut=nodes[nd["parent"]]["cut"], left=-1, right=-1, s1=F(0), s2=F(0))
            rd += 1
            continue
        nd.update(leaf=0, tri=-1, cut=cut)
        left_set = set(lists[cut][l:m + 1])
        for k in range(6):
            if k == cut:
                continue
            seg = lists[k][l:r + 1]
            lists[k][l:r + 1] = [e for e in seg if e in left_set] + [e for e in seg if e not in left_set]
        for br, (nl, nr) in enumerate(((l, m), (m + 1, r))):
            c = dict(l=nl, r=nr, m=(nr - nl) // 2 + nl, parent=rd, x1=key(0, nr), x0=key(3, nl), y1=key(1, nr),
                     y0=key(4, nl), z1=key(2, nr), z0=key(5, nl))
            nd["left" if br == 0 else "right"] = len(nodes)
            nodes.append(c)
        Lc, Rc = nodes[nd["left"]], nodes[nd["right"]]
        ax = "xyz"[cut % 3]
        nd["s1"], nd["s2"] = Lc[ax + "1"], Rc[ax + "0"]
        rd += 1
    return nodes


# -------------------------------------------------------------- render (a3-a8)

def prepare(points9, nodes, cam):
    P = points9.astype(F)
    e1 = (P[:, 3:6] - P[:, 0:3]).astype(F)
    e2 = (P[:, 6:9] - P[:, 0:3]).astype(F)
    nrm = []
    for i in range(len(P)):
        c = cross(e1[i], e2[i])
        nrm.append(dev_normalize(*c))
    pos = cam["pos"]
    dt = np.stack([F(pos[k]) - P[:, k] for k in range(3)], 1).astype(F)
    dq = np.array([cross(dt[i], e1[i]) for i in range(len(P))], F).reshape(-1, 3)
    dw = np.array([dot(dq[i], e2[i]) for i in range(len(P))], F)
    vox = None
    if nodes is not None:
        vox = []
        for nd in nodes:
            c = nd["cut"]
            cf = [F(1) if c in (0, 3) else F(0), F(1) if c in (1, 4) else F(0), F(1) if c in (2, 5) else F(0)]
            bo = [F(F(nd["x0"] - pos[0]) + F(0)), F(F(nd["y0"] - pos[1]) + F(0)), F(F(nd["z0"] - pos[2]) + F(0)),
                  F(F(nd["x1"] - pos[0]) + F(0)), F(F(nd["y1"] - pos[1]) + F(0)), F(F(nd["z1"] - pos[2]) + F(0))]
            sh = F(F(F(F(pos[0] + F(0)) * cf[0]) + F(F(pos[1] + F(0)) * cf[1])) + F(F(pos[2] + F(0)) * cf[2]))
            vox.append(dict(bo=bo, s1=F(F(nd["s1"]) - sh), s2=F(F(nd["s2"]) - sh), leaf=nd["leaf"], tri=nd["tri"],
                            left=nd["left"], right=nd["right"], cf=cf))
    return dict(e1=e1, e2=e2, nrm=np.array(nrm, F), dt=dt, dq=dq, dw=dw, vox=vox)


def _mt_accept(u, v, w, d):
    return (w < d) and not ((D(u) < EPS) or (D(v) < EPS) or (D(F(u + v)) > D(1) + EPS) or (D(w) < EPS))


def _walk(S, r, od, on_leaf, lim=None):
    """The DFS of intersect_voxel_cuda (TD/Trixel.cu:70-170) for direction r and
    translation od; on_leaf(t, u, v, w) sees every non-degenerate MT test.
    lim: a shadow segment's walk enters a box only below lim (oracle.c
    trace_shadow)."""
    inv = [F(F(1) / r[k]) for k in range(3)]
    o = [F(od[k] / r[k]) for k in range(3)]
    stack = [0]
    while stack:
        cni = stack.pop()
        vx = S["vox"][cni]
        if vx["leaf"]:
            t = vx["tri"]
            e1, e2, dt = S["e1"][t], S["e2"][t], S["dt"][t]
            p = cross(r, e2)
            f = dot(p, e1)
            if not (D(f) < EPS and D(f) > -EPS):
                pe1 = F(D(1.0) / D(f))
                tt = [F(dt[k] - od[k]) for k in range(3)]
                u = F(pe1 * dot(p, tt))
                q = cross(tt, e1)
                v = F(pe1 * dot(r, q))
                w = F(pe1 * dot(e2, q))
                on_leaf(t, u, v, w)
            continue
        bo = vx["bo"]
        t0 = [F(bo[k] * inv[k]) if r[k] > 0 else F(bo[k + 3] * inv[k]) for k in range(3)]
        t1 = [F(bo[k + 3] * inv[k]) if r[k] > 0 else F(bo[k] * inv[k]) for k in range(3)]
        cf = vx["cf"]
        dr = F(F(F(r[0] * cf[0]) + F(r[1] * cf[1])) + F(r[2] * cf[2]))
        ds = F(F(F(od[0] * cf[0]) + F(od[1] * cf[1])) + F(od[2] * cf[2]))
        maxt0 = np.fmax(F(t0[2] + o[2]), np.fmax(F(t0[0] + o[0]), F(t0[1] + o[1])))
        mint1 = np.fmin(F(t1[2] + o[2]), np.fmin(F(t1[0] + o[0]), F(t1[1] + o[1])))
        if D(mint1) >= D(maxt0) - EPS and D(maxt0) > -EPS and (lim is None or maxt0 < lim):
            maxt0, mint1 = F(maxt0 * dr), F(mint1 * dr)
            s1 = F(D(vx["s1"]) + EPS + D(ds))
            s2 = F(vx["s2"] + ds)
            if D(maxt0) < D(s2) + EPS:
                if D(mint1) > D(s2) - EPS:
                    stack.append(vx["right"])
                stack.append(vx["left"])
            else:
                if mint1 < s1 or maxt0 < s1:
                    stack.append(vx["left"])
                stack.append(vx["right"])


def trace_kd(S, X, cam_rmd):
    """intersect_voxel_cuda, TD/Trixel.cu:41-172.  Returns (rmi, d, (pnt, nrm),
    (r, od)) -- the last pair is the object-space ray, for the shadow ray."""
    X = [F(x) for x in X]
    od = (X[3], X[7], X[11])
    m = [F(-c) for c in cam_rmd]
    r = [F(F(-1) * F(F(F(X[4 * k] * m[0]) + F(X[4 * k + 1] * m[1])) + F(X[4 * k + 2] * m[2]))) for k in range(3)]
    st = dict(d=F(400.0), rmi=-1, out=None)

    def leaf(t, u, v, w):
        if _mt_accept(u, v, w, st["d"]):
            st["d"], st["rmi"] = w, t
            pnt = [F(F(w * r[k]) + od[k]) for k in range(3)]
            n = S["nrm"][t]
            a = [F(F(-1) * n[k]) for k in range(3)]
            nr = [F(F(F(F(F(a[0] * X[4 * k]) + F(a[1] * X[4 * k + 1])) + F(a[2] * X[4 * k + 2]))) * F(-1))
                  for k in range(3)]
            st["out"] = (pnt, nr)

    _walk(S, r, od, leaf)
    return st["rmi"], st["d"], st["out"], (r, od)


SHADOW_SCALE = F(0.9990234375)  # 1 - 2^-10


def trace_shadow(S, rmi, d, ray, segment=True):
    """The shadow segment of a hit (oracle.c trace_shadow): from the light
    (2,2,2) to H = d*r - od, walked from the light; True if occluded.
    segment=False: rounds 1-5's walk of the whole ray beyond H (tests only:
    the round-6 segment walk gives the same images)."""
    r, od = ray
    sv = [F(F(F(d * r[k]) - od[k]) - F(2)) for k in range(3)]
    L2 = F(F(F(sv[0] * sv[0]) + F(sv[1] * sv[1])) + F(sv[2] * sv[2]))
    lmax = F(F(np.sqrt(D(L2))) * SHADOW_SCALE)
    s = dev_normalize(*sv)
    hit = [False]

    def leaf(t, u, v, w):
        if t != rmi and _mt_accept(u, v, w, lmax):
            hit[0] = True

    _walk(S, list(s), (F(-2), F(-2), F(-2)), leaf, lim=lmax if segment else None)
    return hit[0]


def trace_flat(S, rmd):
    """intersect_trixel_cuda, TD/Trixel.cu:173-209."""
    d, rmi, out = F(400.0), -1, None
    for t in range(len(S["e1"])):
        p = cross(rmd, S["e2"][t])
        f = dot(p, S["e1"][t])
        if not (D(f) < EPS and D(f) > -EPS):
            pe1 = F(D(1.0) / D(f))
            u = F(pe1 * dot(p, S["dt"][t]))
            v = F(pe1 * dot(rmd, S["dq"][t]))
            w = F(pe1 * S["dw"][t])
            if _mt_accept(u, v, w, d):
                d, rmi = w, t
                out = ([F(d * rmd[k]) for k in range(3)], list(S["nrm"][t]))
    return rmi, d, out


def pow5(x):
    dd = D(x)
    d2 = dd * dd
    return F((d2 * d2) * dd)


def to_u8(t):
    if not (t >= 0):
        return 0
    return 255 if t >= 256 else int(t)


def phong(pnt, nrm, rmd, rad):
    """color_cam_cuda, TD/Camera.cu:27-60."""
    sd = dev_normalize(F(F(2) - pnt[0]), F(F(2) - pnt[1]), F(F(2) - pnt[2]))
    dn = dot(sd, (nrm[0], nrm[0], nrm[2]))
    r = [F(F(sd[k] - F(F(F(2) * dn) * nrm[k])) * rmd[k]) for k in range(3)]
    diff = F(0.6 * D(abs(dn)))
    spec = F(D(pow5(abs(F(F(r[0] + r[1]) + r[2])))) * 0.3)
    c = [F(F(0) + F(F(rad[k] * diff) + spec)) for k in range(3)]
    mx = np.fmax(np.fmax(c[0], c[1]), c[2])
    with np.errstate(invalid="ignore", divide="ignore"):
        q = [to_u8(F(F(c[k] / mx) * F(255))) for k in range(3)]
    return (q[0] << 16) | (q[1] << 8) | q[2]


RAD = (F(0.1), F(0.55), F(0.2))


def render(points9, nodes, cam, mode=0, xform=None, shadow=False, segment=True):
    S = prepare(points9, nodes if mode == 0 else None, cam)
    X = IDENT if xform is None else np.asarray(xform, F)
    w, h = cam["w"], cam["h"]
    argb = np.full(w * h, BG, np.uint32)
    hit = np.full(w * h, -1, np.int64)
    with np.errstate(all="ignore"):
        for iy in range(h):
            for ix in range(w):
                rmd = primary_ray(cam, ix, iy)
                if mode == 0:
                    rmi, d, out, ray = trace_kd(S, X, rmd)
                else:
                    rmi, d, out = trace_flat(S, rmd)
                i = iy * w + ix
                hit[i] = rmi
                if rmi >= 0:
                    argb[i] = phong(out[0], out[1], rmd, RAD)
                    if shadow and trace_shadow(S, rmi, d, ray, segment):
                        argb[i] = 0
    return argb, hit


def window_frames(frames, hits):
    """The reference's window across frames (TD/WinMain.cpp:212-237), restated
    independently of oracle.c's orc_window_frame: the buffer starts zeroed
    (TD/Camera.cu:98); color_cam_cuda writes only rmi >= 0 pixels before the
    blit (TD/Camera.cu:27-61); the SET pass leaves background + Phong
    (TD/Camera.cu:77-84).  Returns the displayed frames."""
    buf = np.zeros_like(np.asarray(frames[0], np.uint32))
    out = []
    for argb, hit in zip(frames, hits):
        argb = np.asarray(argb, np.uint32)
        hitm = np.asarray(hit) >= 0
        buf = np.where(hitm, argb, buf)
        out.append(buf.copy())
        buf = np.where(hitm, argb, np.uint32(BG))
    return out
