#!/bin/bash
# A short gpurun session: GPU parity tests, smoke, one default bench line.
# Stops at the first step that faults, aborts or times out.
#   tools/quick_session.sh <tag> [bench args...]
set -u
TAG=${1:-quick}
shift || true
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
step bench 300 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline "$@"
echo "session done"
