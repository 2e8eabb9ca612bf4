#!/bin/bash
# A/B of bench.py argument sets on one box, interleaved ROUNDS times.
#   ARGSETS="--prio 0;--prio 50" tools/args_ab.sh <tag>
set -u
TAG=${1:-args}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
IFS=';' read -r -a SETS <<< "${ARGSETS:-}"
for r in $(seq 1 ${ROUNDS:-2}); do
    i=0
    for a in "${SETS[@]}"; do
        i=$((i + 1))
        log="$OUT/set${i}_$r.log"
        timeout -k 10 200 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline $a > "$log" 2>&1
        rc=$?
        echo "[$a] round $r exit $rc: $(grep -o '"value": [0-9.]*' "$log") $(grep -o '"kernel_ms_avg": [0-9.]*' "$log")"
        if [ $rc -ne 0 ]; then tail -5 "$log"; exit $rc; fi
    done
done
