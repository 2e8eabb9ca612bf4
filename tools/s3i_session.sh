#!/bin/bash
# XCD order before a grid's first cost order: GPU tests, A/B on poses, moving and static bench lines.
set -u
TAG=${1:-s3i}
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
    tail -n 2 "$OUT/$name.log" | cut -c1-300
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name exited $rc"; exit $rc; fi
    return 0
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step xform 300 python tools/exp_xform.py --frames 300 --tile-orders 3 --debug 0,32 --only identity,translate,rotate+translate,moving
step bench_anim 300 python bench.py --steps 500 --warmup 20 --animate R+W.Q.T.W --no-cpu-baseline
step bench_c4 300 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline
step bench_c3 300 python bench.py --width 960 --height 540 --steps 1000 --warmup 100 --no-cpu-baseline
echo "session done"
