#!/bin/bash
# PMC passes (rocprofv3 --pmc, counters only: no trace domains) of the default
# bench workload, summarised into profiles/pmc_traffic.json.
#   tools/pmc_session.sh <tag> [bench args...]
set -u
TAG=${1:-pmc}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
BENCH="bench.py --steps 30 --warmup 5 --no-cpu-baseline $*"
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i + 1))
    timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pass$i" -o run -- python3 $BENCH \
        > "$OUT/pass$i.log" 2>&1
    rc=$?
    echo "pass $i ($ctr) exit $rc"
    if [ $rc -ne 0 ]; then tail -20 "$OUT/pass$i.log"; exit $rc; fi
done
grep -h '^{' "$OUT/pass1.log" | head -1 > "$OUT/bench_line.json"
python3 tools/pmc_traffic.py "${PMC_KEY:-dragon_1920x1080_m0_n1}" "${PMC_KERNEL:-k_trace_kd3<16}" "$OUT"/pass*
