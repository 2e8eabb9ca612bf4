#!/bin/bash
# Build compile-time variants of librt_mi355x.so for A/B runs on one box:
#   tools/build_variants.sh name1:"-DFOO" name2:"-DBAR=3" ...
# -> tools/variants/lib_<name>.so (the product build's sources and flags + extras;
#    tools/bench_variant.py runs bench.py against one)
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/tools/variants"
for v in "$@"; do
    name=${v%%:*}
    defs=${v#*:}
    [ "$defs" = "$v" ] && defs=""
    python3 -m cpp_cuda_raytracer_dev_amd.build --variant "$name" --defs="$defs"
done
ls -la "$ROOT"/tools/variants/*.so
