#!/bin/bash
# Kernel-variant sweep on one GPU: bench.py under each (layout, tile order).
# Usage: tools/bench_sweep.sh <tag> [extra bench args...]
set -u
TAG=${1:-sweep}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for v in "1 0" "2 1" "3 0" "3 1" "3 2"; do
    set -- $v "$@"
    k=$1; o=$2; shift 2
    timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --kernel "$k" --tile-order "$o" "$@" \
        > "$OUT/bench_k${k}_o${o}.log" 2>&1
    rc=$?
    echo "kernel $k order $o exit $rc: $(grep -o '"value": [0-9.]*' "$OUT/bench_k${k}_o${o}.log") $(grep -o '"kernel_ms_avg": [0-9.]*' "$OUT/bench_k${k}_o${o}.log")"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/bench_k${k}_o${o}.log"; exit $rc; fi
done
