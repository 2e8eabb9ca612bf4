#!/bin/bash
# Kernel-3 scheduling experiments: GPU parity (the coarse / cost-order tests
# first, then the rest), bench.py over (tile order, rays per wave, coarse
# groups per wave), then per-wave diagnostics.  Stops at the first step that
# faults or times out.
#   tools/coarse_session.sh <tag>     (VARIANTS="order,rays,coarse ...")
set -u
TAG=${1:-coarse}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
run() {  # run <log> <timeout> <cmd...>
    local log=$1 to=$2
    shift 2
    timeout -k 10 "$to" "$@" > "$OUT/$log" 2>&1
    local rc=$?
    echo "== $log exit $rc"
    if [ $rc -ne 0 ]; then tail -30 "$OUT/$log"; exit $rc; fi
}
if [ -z "${NOTEST:-}" ]; then
    run pytest_new.log 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
        -k "${TESTK:-coarse or cost}" --timeout 300
    tail -2 "$OUT/pytest_new.log"
    run pytest_gpu.log 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300
    tail -2 "$OUT/pytest_gpu.log"
fi
for v in ${VARIANTS:-2,16,0 2,16,8 3,16,8 2,8,8 3,8,8 3,8,0}; do
    IFS=, read -r o r c <<< "$v"
    log="bench_o${o}_r${r}_c${c}.log"
    run "$log" 300 python bench.py --steps 500 --warmup 50 --no-cpu-baseline --tile-order "$o" --rays "$r" --coarse "$c" ${BENCH_ARGS:-}
    echo "order $o rays $r coarse $c: $(grep -o '"value": [0-9.]*' "$OUT/$log") $(grep -o '"kernel_ms_avg": [0-9.]*' "$OUT/$log")"
done
if [ -n "${DIAG:-}" ]; then
    run diag.log 300 python tools/diag_waves.py $DIAG
    tail -1 "$OUT/diag.log"
fi
