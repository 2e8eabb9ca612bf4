#!/bin/bash
# Round-2 measurement session on one GPU: parity tests, smoke, one bench line
# per BASELINE config and view, and rocprofv3 kernel stats of the headline
# and the flat-list (C2) benches.  Stops at the first step that faults,
# aborts or times out (exit codes other than 0, 1 = assertions, 3/4 = bench
# self-check failures, which are reported).
#   tools/r02_session.sh <tag> [steps...]   (steps: tests smoke bench prof; default all)
set -u
TAG=${1:-r02}
shift || true
WANT=${*:-"tests smoke bench prof"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
    local name=$1 to=$2
    shift 2
    echo "== $name: $*"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name exit $rc"
    tail -n 4 "$OUT/$name.log" | cut -c1-600
    case $rc in 0|1|3|4) return 0 ;; esac
    echo "stopping: $name exited $rc"
    exit $rc
}
has() { [[ " $WANT " == *" $1 "* ]]; }
if has tests; then
    step pytest_gpu 1100 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
fi
if has smoke; then
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if has bench; then
    step bench_c4_dragon1080 400 python bench.py --steps 1000 --warmup 100
    step bench_c3_dragon960 300 python bench.py --steps 1000 --warmup 100 --width 960 --height 540 --no-cpu-baseline
    step bench_c2_rabbit_flat 400 python bench.py --scene rabbit_70k --width 960 --height 540 --mode 1 --steps 40 \
        --warmup 4
    step bench_c5_happy4k_shadow 400 python bench.py --steps 200 --warmup 20 --scene happy --width 3840 --height 2160 \
        --shadow --no-cpu-baseline
    step bench_fill_dragon960 300 python bench.py --steps 500 --warmup 50 --width 960 --height 540 --view fill
    step bench_fill_dragon1080 300 python bench.py --steps 300 --warmup 30 --view fill --no-cpu-baseline
    step bench_fill_rabbit1080 300 python bench.py --steps 300 --warmup 30 --scene rabbit_70k --view fill \
        --no-cpu-baseline
    step bench_dragon_shadow 300 python bench.py --steps 500 --warmup 50 --shadow --no-cpu-baseline
    step bench_big 300 python bench.py --steps 200 --warmup 20 --scene big --no-cpu-baseline
    step bench_knot1080 300 python bench.py --steps 1000 --warmup 100 --scene knot --no-cpu-baseline
    step bench_knot960 300 python bench.py --steps 1000 --warmup 100 --scene knot --width 960 --height 540 \
        --no-cpu-baseline
    step bench_knot1080_shadow 300 python bench.py --steps 500 --warmup 50 --scene knot --shadow --no-cpu-baseline
    step bench_rehearse 300 python bench.py --steps 1000 --warmup 100 --rehearse-gather --no-cpu-baseline
    step bench_animate 300 python bench.py --steps 500 --warmup 20 --animate R+W.Q.T.W --no-cpu-baseline
fi
if has prof; then
    step rocprof_c4 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4" -o run -- \
        python3 bench.py --steps 1000 --warmup 100 --no-cpu-baseline
    step rocprof_c4_solo 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4_solo" -o run -- \
        python3 bench.py --steps 1000 --warmup 100 --no-cpu-baseline --inflight 1
    step rocprof_c2 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o run -- \
        python3 bench.py --scene rabbit_70k --width 960 --height 540 --mode 1 --steps 20 --warmup 2 --no-cpu-baseline
fi
echo "session done"
