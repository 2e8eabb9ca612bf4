#!/bin/bash
# Unrolled certain-miss pass of the coarse kernel: parity, transform poses, kernel breakdown, moving bench.
set -u
TAG=${1:-s3g}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
    local name=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name exit $rc"
    tail -n 3 "$OUT/$name.log" | cut -c1-400
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name exited $rc"; exit $rc; fi
    return 0
}
step pytest_coarse 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "coarse or transform or poses or animat or motion or key"
step xform 300 python tools/exp_xform.py --frames 300 --tile-orders 3
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 tools/exp_xform.py --frames 300 --tile-orders 3 --only translate,moving
step bench_anim 300 python bench.py --steps 500 --warmup 20 --animate R+W.Q.T.W --no-cpu-baseline
echo "session done"
