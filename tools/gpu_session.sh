#!/bin/bash
# One gpurun session: GPU parity tests -> smoke -> bench -> rocprofv3 stats.
# Stops at the first step that faults, aborts or times out (exit codes other
# than 0 = pass and 1 = test assertions failed).  Usage (from the repo root):
#   tools/gpu_session.sh <tag> [pytest-args...]
set -u
TAG=${1:-r01}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"

step() {  # step <name> <timeout> <cmd...>
    local name=$1 to=$2
    shift 2
    echo "== $name: $*" | tee -a "$OUT/session.log"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name exit $rc" | tee -a "$OUT/session.log"
    tail -n 25 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping: $name exited $rc" | tee -a "$OUT/session.log"
        exit $rc
    fi
    return $rc
}

step pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider "$@"
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py --steps 500 --warmup 50
export TMPDIR=/tmp
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 500 --warmup 50 --no-cpu-baseline
echo "session done" | tee -a "$OUT/session.log"
