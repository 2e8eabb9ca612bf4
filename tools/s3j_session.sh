#!/bin/bash
# Whole-frame order slots / cost buffers: GPU tests, held-pose sequence, moving bench.
set -u
TAG=${1:-s3j}
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
step hold 400 python tools/exp_xform.py --frames 640 --tile-orders 3 --holds 1,2,4,8,32 --only identity,moving,moving_hold2,moving_hold4,moving_hold8,moving_hold32
step bench_anim 300 python bench.py --steps 500 --warmup 20 --animate R+W.Q.T.W --no-cpu-baseline
step bench_anim1k 300 python bench.py --steps 1000 --warmup 20 --animate R+W.Q.T.W --no-cpu-baseline
echo "session done"
