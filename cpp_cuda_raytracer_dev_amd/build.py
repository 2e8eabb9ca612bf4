"""Build the in-tree HIP library (gfx950) and the headless driver.

    python -m cpp_cuda_raytracer_dev_amd.build            # librt_mi355x.so
    python -m cpp_cuda_raytracer_dev_amd.build --driver   # + tools/rt_headless

Flags that are part of the parity contract:
-ffp-contract=off (no FMA contraction), correctly rounded fp32 division,
f32 denormals kept.  No fast-math.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "librt_mi355x.so")
ARCH = os.environ.get("RT_OFFLOAD_ARCH", "gfx950")

# (source, object name, extra flags): rt_kd_dispatch.hip is compiled once per
# (translated, write-hit, count) combination, so the KD kernels' template
# instances build in parallel
SOURCES = [("rt_kernels.hip", "rt_kernels", [])] + [
    ("rt_kd_dispatch.hip", f"rt_kd_{t}{h}{c}", [f"-DRT_KD_T={t}", f"-DRT_KD_H={h}", f"-DRT_KD_C={c}"])
    for t in (0, 1) for h in (0, 1) for c in (0, 1)] + [
    (f, os.path.splitext(f)[0], []) for f in ("kd_build_gpu.hip", "rt_api.cpp", "scene_host.cpp", "motion.cpp", "comm.cpp")]
OBJ = os.path.join(PKG, "_obj")  # per-source objects (git- and gpurun-ignored)
# -fno-slp-vectorize: hipcc's packed-math (v_pk_*) SLP pairs cost more register
# moves than they save in the traversal loop (0.0851 vs 0.0871 ms per 1080p
# dragon frame); the arithmetic per lane is the same IEEE operations either way.
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
             "-fno-gpu-flush-denormals-to-zero", "-fno-slp-vectorize", "-Wall", f"--offload-arch={ARCH}"]


def hipcc() -> str:
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_lib(force: bool = False, verbose: bool = False, jobs: int = 0, out: str = LIB, defs=(),
              objdir: str = OBJ) -> str:
    """Compile each source to its own object (only the stale ones, in
    parallel), then link.  out / defs / objdir: an experiment variant (extra
    -D flags, its own objects), e.g. tools/build_variants.sh."""
    from concurrent.futures import ThreadPoolExecutor
    headers = [os.path.join(CSRC, h) for h in ("rt_internal.h", "rt_predicates.h", "rt_kernels_impl.h")] + [
        os.path.join(ROOT, "include", "rt_mi355x.h")]
    os.makedirs(objdir, exist_ok=True)
    objs, todo = [], []
    relink = force or not os.path.exists(out)
    for src, name, extra in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(objdir, name + ".o")
        objs.append(obj)
        if force or _stale(obj, [path, *headers, __file__]):
            todo.append(([hipcc(), *HIP_FLAGS, *defs, *extra, "-c", "-o", obj + ".tmp", path], obj))

    def compile_one(job):
        cmd, obj = job
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(obj + ".tmp", obj)

    if todo:
        n = jobs or min(len(todo), max(1, len(os.sched_getaffinity(0))), 16)
        with ThreadPoolExecutor(n) as ex:
            list(ex.map(compile_one, todo))
        relink = True
    if not relink and not _stale(out, objs):
        return out
    tmp = out + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-o", tmp, *objs, "-lpthread", "-ldl"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


def build_driver(verbose: bool = False) -> str:
    src = os.path.join(ROOT, "tools", "rt_headless.cpp")
    out = os.path.join(ROOT, "tools", "rt_headless")
    if not os.path.exists(src):
        return ""
    if _stale(out, [src, LIB, os.path.join(ROOT, "include", "rt_facade.hpp")]):
        cmd = ["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-o", out, src, LIB,
               f"-Wl,-rpath,{PKG}", "-lpthread"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--driver", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--variant", default="", help="experiment build: tools/variants/lib_<name>.so")
    ap.add_argument("--defs", default="", help="extra compile flags of the variant, e.g. '-DRT_POOL_CAP_R16=384'")
    a = ap.parse_args(argv)
    if a.variant:
        vdir = os.path.join(ROOT, "tools", "variants")
        print(build_lib(a.force, a.verbose, out=os.path.join(vdir, f"lib_{a.variant}.so"), defs=a.defs.split(),
                        objdir=os.path.join(vdir, "_obj_" + a.variant)))
        return 0
    print(build_lib(a.force, a.verbose))
    if a.driver:
        print(build_driver(a.verbose))
    return 0


if __name__ == "__main__":
    sys.exit(main())
