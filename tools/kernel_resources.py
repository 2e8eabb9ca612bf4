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


def occupancy(cur):
    """Waves per SIMD of a k_trace_kd3 instance: by VGPRs (allocation granule
    8, 512 per SIMD lane, at most 8: MI355X_MICROARCH.md register files) and
    by LDS (160 KiB per CU, the block's waves spread over 4 SIMDs); the
    smaller binds.  Other kernels: the VGPR bound only."""
    alloc = -(-int(cur[".vgpr_count"]) // 8) * 8
    by_vgpr = min(8, 512 // max(alloc, 8))
    m = re.search(r"k_trace_kd3ILi(\d+)E", cur[".name"])
    lds = int(cur[".group_segment_fixed_size"])
    if not m or lds == 0:
        return f"waves/SIMD {by_vgpr} (vgpr)"
    waves_per_block = 4 if int(m.group(1)) <= 16 else 2
    by_lds = (160 * 1024 // lds) * waves_per_block // 4
    return f"waves/SIMD {min(by_vgpr, by_lds)} (vgpr {by_vgpr}, lds {by_lds})"


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
                              f"scratch {cur['.private_segment_fixed_size']:>4}  {occupancy(cur)}  {cur['.name']}")
                    cur = {}


if __name__ == "__main__":
    main()
