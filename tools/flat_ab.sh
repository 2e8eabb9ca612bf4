#!/bin/bash
# Flat-list kernel forms A/B on C2 (rabbit_70k 960x540), after the GPU tests.
#   tools/flat_ab.sh <tag> [forms...]
set -u
TAG=${1:-flat}
shift || true
FORMS=${*:-2 4 5}
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
    tail -n 2 "$OUT/$name.log" | cut -c1-400
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name exited $rc"; exit $rc; fi
    return 0
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
for f in $FORMS; do
    step "c2_form$f" 200 python bench.py --scene rabbit_70k --width 960 --height 540 --mode 1 --flat "$f" \
        --steps 60 --warmup 5 --no-cpu-baseline
done
echo "session done"
