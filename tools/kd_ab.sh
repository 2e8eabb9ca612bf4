#!/bin/bash
# After a kernel-3 change: the GPU tests, then C4, C3, the 1080p fill view and
# the knot at 1080p (no CPU baseline).  Stops at the first fault or timeout.
set -u
TAG=${1:-kd_ab}
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
    tail -n 1 "$OUT/$name.log" | cut -c1-200
    case $rc in 0|1|3|4) return 0 ;; esac
    echo "stopping: $name exited $rc"; exit $rc
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step c4 300 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline
step c3 300 python bench.py --steps 1000 --warmup 100 --width 960 --height 540 --no-cpu-baseline
step fill1080 300 python bench.py --steps 300 --warmup 30 --view fill --no-cpu-baseline
step knot1080 300 python bench.py --steps 1000 --warmup 100 --scene knot --no-cpu-baseline
step c5 300 python bench.py --steps 200 --warmup 20 --scene happy --width 3840 --height 2160 --shadow --no-cpu-baseline
echo "session done"
