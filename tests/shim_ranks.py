"""N ranks of the multi-GPU frame loop as threads of one process on one GPU
(VERDICT r03 item 4).  TEST DRIVER: run by tests/test_gpu_parity.py::
test_shim_ranks_gather in a child process whose environment sets RT_RCCL_LIB
to tests/rccl_shim/librccl_shim.so, the test-only in-process RCCL stand-in.

Each rank r of N is a thread with its own rt_camera (device 0), its own
rt_comm (rt_comm_create through the shim) and streams, and renders its
interleaved 8-row bands with rt_run_frames exactly as bench.py does at N > 1:
two frames in flight on the camera's lanes, four buffer sets, the gather on
the comm lane (csrc/comm.cpp: the peers' k_pack_rect + ncclSend, rank 0's
ncclRecv loop and k_unpack_rect), rank 0 rendering straight into its frame
(RT_FLAG_FRAME_OUT), one object pose per frame (rt_frame_loop.xforms).  The
threads call into the library concurrently (ctypes drops the GIL).

After the loop every buffer set of rank 0 holds the frame of its last use;
each is compared with the oracle: the committed full-frame hash for the
identity pose (tests/golden/frame_hashes.json) and a live oracle render for
the moved poses.  Prints one JSON line; exit status 0 iff every frame matches
and every rank's device error word is 0.

    RT_RCCL_LIB=tests/rccl_shim/librccl_shim.so python tests/shim_ranks.py \
        --nranks 2,4,8 --scene dragon --width 1920 --height 1080 --frames 24
"""
import argparse
import hashlib
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class ThreadGroup:
    """What NativeFrameGather needs of torch.distributed, for threads: the
    RCCL id broadcast and the agreement check (all_gather_object)."""

    def __init__(self, n):
        self.n = n
        self.bar = threading.Barrier(n, timeout=60)
        self.box = {}


class ThreadDist:
    def __init__(self, grp, rank):
        self.grp, self.rank = grp, rank

    def get_rank(self):
        return self.rank

    def get_world_size(self):
        return self.grp.n

    def barrier(self):
        self.grp.bar.wait()

    def broadcast_object_list(self, objs, src=0):
        if self.rank == src:
            self.grp.box["bcast"] = list(objs)
        self.grp.bar.wait()
        objs[:] = self.grp.box["bcast"]
        self.grp.bar.wait()

    def all_gather_object(self, out, obj):
        self.grp.box[("ag", self.rank)] = obj
        self.grp.bar.wait()
        out[:] = [self.grp.box[("ag", r)] for r in range(self.grp.n)]
        self.grp.bar.wait()


def rot_y_xform(deg, t=(0.0, 0.0, 0.0)):
    """A rot_m (3x4 rows, float32) turning the object by `deg` about y, offset t."""
    a = np.deg2rad(np.float64(deg))
    c, s = np.float32(np.cos(a)), np.float32(np.sin(a))
    return np.array([[c, 0, s, t[0]], [0, 1, 0, t[1]], [-s, 0, c, t[2]]], np.float32).reshape(12)


POSES = [rot_y_xform(0.0), rot_y_xform(3.0), rot_y_xform(0.0, (0.01, 0.0, 0.0)), rot_y_xform(-4.0),
         rot_y_xform(1.5, (0.0, 0.004, 0.0))]


def run_group(n, scene, w, h, frames, inflight, nbuf, trixel, oracle_frame, poses, flags):
    import torch
    from cpp_cuda_raytracer_dev_amd import raytracer as R, scenes
    from cpp_cuda_raytracer_dev_amd.distributed import NativeFrameGather
    dev = torch.device("cuda", 0)
    grp = ThreadGroup(n)
    cam_kw = scenes.view(scene, "default")
    state = [dict() for _ in range(n)]
    errors = []

    def rank_main(r):
        try:
            st = state[r]
            d = ThreadDist(grp, r)
            cam = R.Camera(w, h, R.film_w(w, h), np.float32(.024), np.float32(.055), *cam_kw["pos"],
                           *cam_kw["look_at"], 0.0, 1.0, 0.0, device=0)
            obj = R.Object(trixel)
            cam.add_object(obj)
            ng = NativeFrameGather(d, w, h, dev, nbuf=nbuf)
            for f in ng.frames:  # poisoned: a row nobody wrote shows
                if f is not None:
                    f.fill_(0x7BADBEEF)
            for loc in ng.local:
                loc.fill_(0x5EEDF00D)
            rect = ng.verify(cam, None, 0)
            rs, cs = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
            loop = R.FrameLoop(cam, ng.local, mode=0, flags=flags, tile=(n, r), render_stream=rs.cuda_stream,
                               comm=ng, comm_stream=cs.cuda_stream, event_every=8, inflight=inflight,
                               xforms=np.stack(poses))
            torch.cuda.synchronize(dev)
            d.barrier()
            t0 = time.perf_counter()
            loop.run(frames)
            st["seconds"] = time.perf_counter() - t0
            torch.cuda.synchronize(dev)
            st.update(cam=cam, obj=obj, ng=ng, loop=loop, rect=rect, err=cam.device_error(reset=True))
        except BaseException as e:  # noqa: BLE001 -- reported, the process exits non-zero
            errors.append(f"rank {r}: {type(e).__name__}: {e}")
            os._exit(5)  # peers may be blocked in the shim's rendezvous: end the process

    threads = [threading.Thread(target=rank_main, args=(r,), daemon=True) for r in range(n)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=90)
    if any(t.is_alive() for t in threads) or errors:
        print(json.dumps({"nranks": n, "ok": False, "errors": errors or ["a rank did not finish in 90 s"]}),
              flush=True)
        os._exit(6)
    ng0 = state[0]["ng"]
    sets = []
    ok = True
    for k in range(nbuf):
        j = max(i for i in range(frames) if i % nbuf == k)  # the set's last frame
        p = j % len(poses)
        got = ng0.frames[k].cpu().numpy().view(np.uint32)
        ref, how = oracle_frame(p)  # a frame, or the SHA-256 of one
        sha = hashlib.sha256(got.tobytes()).hexdigest()
        same = sha == ref if isinstance(ref, str) else bool(np.array_equal(got, ref))
        ok = ok and same
        sets.append({"set": k, "frame": j, "pose": p, "equal": same, "method": how, "sha256": sha[:16],
                     "diff_pixels": None if isinstance(ref, str) else int((got != ref).sum())})
    errs = [int(s["err"]) for s in state]
    ok = ok and not any(errs)
    out = {"nranks": n, "ok": ok, "device_err": errs, "frames": frames, "inflight": inflight, "nbuf": nbuf,
           "rect_identity": list(state[0]["rect"]), "sets": sets,
           "seconds_per_rank": [round(s["seconds"], 4) for s in state]}
    for s in state:  # explicit release, in dependency order
        for k in ("ng", "cam"):
            s[k].close()
        s["obj"].motion.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nranks", default="2,4,8")
    ap.add_argument("--scene", default="dragon")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--inflight", type=int, default=2)
    ap.add_argument("--nbuf", type=int, default=4)
    ap.add_argument("--shadow", action="store_true", help="one shadow ray per hit (config C5)")
    ap.add_argument("--identity-only", action="store_true", help="every frame at the identity pose")
    a = ap.parse_args()
    if not os.environ.get("RT_RCCL_LIB"):
        print("shim_ranks.py: RT_RCCL_LIB must name tests/rccl_shim/librccl_shim.so", file=sys.stderr)
        return 2
    import torch  # noqa: F401  (its HIP runtime first, as _lib requires)
    from cpp_cuda_raytracer_dev_amd import _lib, raytracer as R, scenes
    from oracle import _oracle as O
    from tests import helpers as H
    assert _lib.lib().rt_comm_available() == 1, "the shim did not load"
    w, h = a.width, a.height
    pts, leafs, _ = H.mesh(a.scene)
    nodes = H.product_tree(a.scene)  # byte-equal to the oracle's create_kd (tests/test_host_cpu.py)
    trixel = R.Trixel(len(pts), pts, device=0)
    trixel.set_kd_nodes(nodes)
    cam_kw = scenes.view(a.scene, "default")
    ent = H.frame_hashes().get(f"{a.scene}_{w}x{h}_m0" + ("_shadow" if a.shadow else ""))
    poses = POSES[:1] if a.identity_only else POSES
    flags = R.RT_FLAG_SHADOW if a.shadow else 0
    cache = {}

    def oracle_frame(p):
        """Pose p's frame: the committed hash (identity pose), else an oracle render."""
        if p not in cache:
            if p == 0 and ent is not None and H.mesh_matches(ent):
                cache[p] = (ent["argb_sha"], "sha256 vs tests/golden/frame_hashes.json")
            else:
                on = np.zeros(len(nodes), O.NODE_DTYPE)
                for k in nodes.dtype.names:
                    on[k] = nodes[k]
                s = O.Scene(pts, O.default_rad(len(pts)), on, O.camera(w, h, **cam_kw))
                ref, _, _ = s.render(0, xform=poses[p].reshape(3, 4), nthreads=H.ORACLE_THREADS, want_hit=False,
                                     shadow=a.shadow)
                s.close()
                cache[p] = (ref, "oracle render at the pose")
        return cache[p]

    results = [run_group(int(n), a.scene, w, h, a.frames, a.inflight, a.nbuf, trixel, oracle_frame, poses, flags)
               for n in a.nranks.split(",")]
    trixel.close()
    ok = all(r["ok"] for r in results)
    print(json.dumps({"ok": ok, "scene": a.scene, "resolution": [w, h], "shadow": a.shadow, "build_id": _lib.build_id(),
                      "rccl": os.environ["RT_RCCL_LIB"], "groups": results}), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
