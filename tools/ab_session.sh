#!/bin/bash
# A/B of library variants (tools/variants/lib_*.so) on one box: bench.py under
# each, interleaved ROUNDS times so box drift hits every variant alike.
#   tools/ab_session.sh <tag> [bench args...]      (VARIANTS="a b ...", ROUNDS=2)
set -u
TAG=${1:-ab}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for r in $(seq 1 ${ROUNDS:-2}); do
    for v in ${VARIANTS:-$(ls tools/variants | sed -n 's/^lib_\(.*\)\.so$/\1/p')}; do
        log="$OUT/${v}_$r.log"
        timeout -k 10 200 python tools/bench_variant.py "tools/variants/lib_$v.so" --steps 1000 --warmup 100 \
            --no-cpu-baseline "$@" > "$log" 2>&1
        rc=$?
        echo "$v round $r exit $rc: $(grep -o '"value": [0-9.]*' "$log") $(grep -o '"kernel_ms_avg": [0-9.]*' "$log")"
        if [ $rc -ne 0 ]; then tail -5 "$log"; exit $rc; fi
    done
done
