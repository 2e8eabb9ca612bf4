#!/bin/bash
# End-of-session check on the final build: GPU tests, smoke, every BASELINE
# config's bench line, the rehearsed N>1 loop, rocprof of the solo C4 frames.
set -u
TAG=${1:-s3final}
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
step bench_c4 300 python bench.py --steps 1000 --warmup 100
step bench_c3 300 python bench.py --width 960 --height 540 --steps 1000 --warmup 100 --no-cpu-baseline
step bench_c5 300 python bench.py --scene happy --width 3840 --height 2160 --shadow --steps 300 --warmup 30 --no-cpu-baseline
step bench_c2 300 python bench.py --scene rabbit_70k --width 960 --height 540 --mode 1 --steps 100 --warmup 5 --no-cpu-baseline
step rehearse 300 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline --rehearse-gather
step prof_c4_solo 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4_solo" -o run -- \
    python3 bench.py --steps 1000 --warmup 100 --no-cpu-baseline --inflight 1
echo "session done"
