#!/bin/bash
# Round-2 third-session check: GPU tests, smoke, the C4 line, and the
# moving-object kernel breakdown (one frame in flight, rocprofv3 stats).
# Stops at the first step that faults, aborts or times out.
set -u
TAG=${1:-s3}
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
    tail -n 3 "$OUT/$name.log" | cut -c1-600
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name exited $rc"; exit $rc; fi
    return 0
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c4 300 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline
step anim_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/anim_prof" -o run -- \
    python3 bench.py --steps 500 --warmup 20 --animate R+W.Q.T.W --no-cpu-baseline --inflight 1
echo "session done"
