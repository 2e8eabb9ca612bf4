#!/bin/bash
# Kernel-variant sweep on one GPU: bench.py under each (kernel, tile order,
# rays per wave).  Usage: tools/bench_sweep.sh <tag> [extra bench args...]
set -u
TAG=${1:-sweep}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
VARIANTS=${VARIANTS:-"2,1,64 3,2,64 3,1,32 3,2,32 3,1,16 3,2,16"}
for v in $VARIANTS; do
    IFS=, read -r k o r <<< "$v"
    log="$OUT/bench_k${k}_o${o}_r${r}.log"
    timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --kernel "$k" --tile-order "$o" \
        --rays "$r" "$@" > "$log" 2>&1
    rc=$?
    echo "kernel $k order $o rays $r exit $rc: $(grep -o '"value": [0-9.]*' "$log") $(grep -o '"kernel_ms_avg": [0-9.]*' "$log")"
    if [ $rc -ne 0 ]; then tail -5 "$log"; exit $rc; fi
done
