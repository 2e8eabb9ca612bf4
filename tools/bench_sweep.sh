#!/bin/bash
# Kernel-variant sweep on one GPU: bench.py under each (kernel, tile order,
# rays per wave, items per lane).  Usage: tools/bench_sweep.sh <tag> [extra bench args...]
set -u
TAG=${1:-sweep}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
VARIANTS=${VARIANTS:-"2,1,64,1 3,2,64,2 3,2,32,1 3,2,32,2 3,2,16,2"}
for v in $VARIANTS; do
    IFS=, read -r k o r i <<< "$v"
    i=${i:-2}
    log="$OUT/bench_k${k}_o${o}_r${r}_i${i}.log"
    timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --kernel "$k" --tile-order "$o" \
        --rays "$r" --items "$i" "$@" > "$log" 2>&1
    rc=$?
    echo "kernel $k order $o rays $r items $i exit $rc: $(grep -o '"value": [0-9.]*' "$log") $(grep -o '"kernel_ms_avg": [0-9.]*' "$log")"
    if [ $rc -ne 0 ]; then tail -5 "$log"; exit $rc; fi
done
