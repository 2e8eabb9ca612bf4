#!/bin/bash
# Kernel breakdown of the moving-object bench (one frame in flight).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-anim_prof}
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 500 --warmup 20 --animate R+W.Q.T.W --no-cpu-baseline --inflight 1 > "$OUT/bench.log" 2>&1
echo "rc $?"
grep '^{' "$OUT/bench.log" | cut -c1-300
