#!/bin/bash
# Average resident waves of one kernel (SQ_LEVEL_WAVES / SQ_BUSY_CYCLES) for
# the given bench.py arguments, one frame in flight.
#   tools/pmc_occ.sh <tag> [bench args...]
set -u
OUT=gpurun_out/${1:-pmc_occ}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LEVEL_WAVES SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv \
    -d "$OUT/occ" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --inflight 1 "$@" > "$OUT/occ.log" 2>&1
echo "exit $?"
