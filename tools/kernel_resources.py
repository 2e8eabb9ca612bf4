#!/usr/bin/env python3
"""Register / LDS / spill figures of the gfx950 kernels in a built library:
splits the .hip_fatbin section into its offload bundles, unbundles each
gfx950 code object and reads its AMDGPU metadata notes.

    python tools/kernel_resources.py [lib.so] [--match k_trace_kd3]
"""
import argparse
import os
import re
import struct
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib):
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(d, "x")],
                       check=True)
        data = open(fat, "rb").read()
        for k, m in enumerate(re.finditer(re.escape(MAGIC), data)):
            base = m.start()
            n = struct.unpack_from("<Q", data, base + len(MAGIC))[0]
            off = base + len(MAGIC) + 8
            for _ in range(n):
                o, size, tlen = struct.unpack_from("<QQQ", data, off)
                triple = data[off + 24:off + 24 + tlen].decode()
                off += 24 + tlen
                if "gfx950" in triple and size:
                    yield data[base + o:base + o + size]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                          "cpp_cuda_raytracer_dev_amd", "librt_mi355x.so"))
    ap.add_argument("--match", default="k_trace_kd3")
    a = ap.parse_args()
    fields = (".name", ".vgpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
              ".group_segment_fixed_size", ".private_segment_fixed_size")
    with tempfile.TemporaryDirectory() as d:
        for k, co in enumerate(code_objects(a.lib)):
            p = os.path.join(d, f"co{k}")
            open(p, "wb").write(co)
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", p], capture_output=True, text=True).stdout
            cur = {}
            for line in notes.splitlines():
                line = line.strip().lstrip("- ").strip()
                for f in fields:
                    if line.startswith(f + ":"):
                        cur[f] = line.split(":", 1)[1].strip()
                if len(cur) == len(fields):
                    if a.match in cur[".name"]:
                        print(f"vgpr {cur['.vgpr_count']:>4} sgpr {cur['.sgpr_count']:>4} spill v{cur['.vgpr_spill_count']}"
                              f"/s{cur['.sgpr_spill_count']} lds {cur['.group_segment_fixed_size']:>6} "
                              f"scratch {cur['.private_segment_fixed_size']:>4}  {cur['.name']}")
                    cur = {}


if __name__ == "__main__":
    main()
