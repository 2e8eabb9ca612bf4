#!/bin/bash
# SQ counter passes of the flat kernel (C2) for the given forms.
set -u
OUT=gpurun_out/${1:-pmc_flat}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for f in "$@"; do
  i=0
  for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
             "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/f${f}_pass$i" -o run -- python3 bench.py \
        --scene rabbit_70k --width 960 --height 540 --mode 1 --flat $f --steps 3 --warmup 1 --no-cpu-baseline --inflight 1 \
        > "$OUT/f${f}_pass$i.log" 2>&1
    rc=$?
    echo "form $f pass $i exit $rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/f${f}_pass$i.log"; exit $rc; fi
  done
done
