#!/bin/bash
# Build compile-time variants of librt_mi355x.so for A/B runs on one box:
#   tools/build_variants.sh name1:"-DFOO" name2:"-DBAR=3" ...
# -> tools/variants/lib_<name>.so (same flags as the product build + extras)
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/tools/variants"
rm -f "$ROOT"/tools/variants/lib_*.so  # only this build's variants travel
FLAGS=$(python3 -c "import sys; sys.path.insert(0, '$ROOT'); from cpp_cuda_raytracer_dev_amd import build as B; print(' '.join(B.HIP_FLAGS))")
SRC="$ROOT/cpp_cuda_raytracer_dev_amd/csrc"
for v in "$@"; do
    name=${v%%:*}
    defs=${v#*:}
    [ "$defs" = "$v" ] && defs=""
    /opt/rocm/bin/hipcc $FLAGS $defs -shared -o "$ROOT/tools/variants/lib_$name.so" \
        "$SRC/rt_kernels.hip" "$SRC/rt_api.cpp" "$SRC/scene_host.cpp" "$SRC/motion.cpp" -lpthread &
done
wait
ls -la "$ROOT/tools/variants"
