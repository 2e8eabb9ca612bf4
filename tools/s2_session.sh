#!/bin/bash
# Round-2 second-session check: GPU tests, smoke, C4 (N=1), the rehearsed
# multi-GPU loop, C2 (flat).  Stops at the first step that faults or times out.
set -u
TAG=${1:-s2}
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
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c4 300 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline
step rehearse 300 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline --rehearse-gather
step bench_c2 300 python bench.py --scene rabbit_70k --width 960 --height 540 --mode 1 --steps 100 --warmup 5 --no-cpu-baseline
echo "session done"
