#!/bin/bash
# The round's measurement session on one GPU: parity tests, smoke, the
# default bench (with the CPU baseline), its rocprofv3 kernel stats, the PMC
# traffic passes, and the secondary configs (C3 960x540, dragon + shadow,
# C5 happy 4K + shadow).  Stops at the first step that faults or times out.
#   tools/round_session.sh <tag>
set -u
TAG=${1:-round}
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
    tail -n 3 "$OUT/$name.log" | cut -c1-400
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name exited $rc"; exit $rc; fi
    return 0
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py --steps 1000 --warmup 100
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 1000 --warmup 100 --no-cpu-baseline
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i + 1))
    step "pmc$i" 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc$i" -o run -- \
        python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline
done
step bench_c3_960x540 300 python bench.py --steps 1000 --warmup 100 --width 960 --height 540 --no-cpu-baseline
step bench_dragon_shadow 300 python bench.py --steps 500 --warmup 50 --shadow --no-cpu-baseline
step bench_happy_shadow 300 python bench.py --steps 500 --warmup 50 --scene happy --shadow --no-cpu-baseline
step bench_animate 300 python bench.py --steps 1000 --warmup 100 --animate "R+W.Q.T.W" --no-cpu-baseline
step bench_c5_happy4k_shadow 400 python bench.py --steps 200 --warmup 20 --scene happy --width 3840 --height 2160 \
    --shadow --no-cpu-baseline
echo "session done"
