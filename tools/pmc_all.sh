#!/bin/bash
# All PMC passes for one bench.py configuration (rocprofv3 --pmc, counters
# only, one pass per counter group, each under its own time limit), then one
# summary entry in profiles/pmc_traffic.json: HBM-side bytes (FETCH_SIZE x2
# on gfx950 + WRITE_SIZE), L2 hit rate, the SQ wave-time split and the L1
# miss latency.
#   tools/pmc_all.sh <tag> <key> <kernel-substring> [bench args...]
set -u
TAG=$1; KEY=$2; KSUB=$3
shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --steps 30 --warmup 5 --no-cpu-baseline --inflight 1 $*"
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pass$i" -o run -- python3 $BENCH \
        > "$OUT/pass$i.log" 2>&1
    rc=$?
    echo "pass $i ($ctr) exit $rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/pass$i.log"; exit $rc; fi
done
python3 tools/pmc_traffic.py "$KEY" "$KSUB" "$OUT"/pass*
