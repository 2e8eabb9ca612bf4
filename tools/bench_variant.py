"""Run bench.py against an alternative build of the library (experiments:
compile-time variants such as pool capacities).  Usage:
    python tools/bench_variant.py <path/to/librt_mi355x.so> [bench args...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    from cpp_cuda_raytracer_dev_amd import _lib
    _lib.LIB_PATH = os.path.abspath(sys.argv[1])
    sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
    import bench
    sys.exit(bench.main())
