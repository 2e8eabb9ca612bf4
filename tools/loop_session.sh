#!/bin/bash
# Frame-loop check: the loop / gather GPU tests, then C4 at N=1 and the
# rehearsed multi-GPU loop, alternating.  Stops at the first fault or timeout.
set -u
TAG=${1:-loop}
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
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name exited $rc"; exit $rc; fi
    return 0
}
step pytest_loop 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "native or rect or frame_loop or frame_out or comm or gather"
for i in 1 2; do
    step "c4_$i" 300 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline
    step "rehearse_$i" 300 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline --rehearse-gather
done
echo "session done"
