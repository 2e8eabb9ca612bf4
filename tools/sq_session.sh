#!/bin/bash
# SQ (wave-state) and HBM-traffic counters of the default bench workload, one
# rocprofv3 --pmc pass per counter group (counters only, no trace domains).
#   tools/sq_session.sh <tag> [bench args...]
set -u
TAG=${1:-sq}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
BENCH="bench.py --steps 30 --warmup 5 --no-cpu-baseline $*"
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA" \
           ${PMC_EXTRA:-}; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/sq$i" -o run -- python3 $BENCH \
        > "$OUT/sq$i.log" 2>&1
    rc=$?
    echo "pass $i ($ctr) exit $rc"
    if [ $rc -ne 0 ]; then tail -20 "$OUT/sq$i.log"; exit $rc; fi
done
python3 tools/pmc_summary.py "$OUT"/sq*
