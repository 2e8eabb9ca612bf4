#!/bin/bash
# Frames in flight A/B for the small frame (C3) and the headline (C4).
set -u
TAG=${1:-s3f}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
for cfg in "c3 --width 960 --height 540" "c4 --width 1920 --height 1080"; do
  set -- $cfg; name=$1; shift
  for L in 2 3 4; do
    timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline --inflight $L "$@" > "$OUT/${name}_L$L.log" 2>&1
    rc=$?
    echo "== $name L=$L exit $rc"; grep '^{' "$OUT/${name}_L$L.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['frame_check']['matches_oracle'], d['device_err'])"
    [ $rc -ne 0 ] && exit $rc
  done
done
echo "session done"
