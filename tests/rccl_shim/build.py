"""Build the TEST-ONLY RCCL stand-in (rccl_shim.cpp -> librccl_shim.so, gfx950
host code; hipcc links the HIP runtime).  Used by tests/shim_ranks.py through
RT_RCCL_LIB; never by the product."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "rccl_shim.cpp")
LIB = os.path.join(HERE, "librccl_shim.so")


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        cmd = ["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "--offload-arch=gfx950",
               "-o", LIB + ".tmp", SRC, "-lpthread"]
        subprocess.run(cmd, check=True)
        os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build("--force" in sys.argv))
