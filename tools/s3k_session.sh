#!/bin/bash
# Same-box A/B of the moving-object bench: whole-frame buffers (default) vs
# current-grid sizing (debug 64).
set -u
TAG=${1:-s3k}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
for rep in 1 2; do
for d in 0 64; do
  timeout -k 10 200 python bench.py --steps 500 --warmup 20 --animate R+W.Q.T.W --no-cpu-baseline --debug-bits $d > "$OUT/anim_d${d}_r$rep.log" 2>&1
  rc=$?
  echo "== debug $d rep $rep exit $rc"; grep '^{' "$OUT/anim_d${d}_r$rep.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], r['kernel_ms_avg'], r['kernel_ms_avg_timed'], d['host']['us_per_frame'], d['frame_check']['matches_oracle'], d['device_err'])"
  [ $rc -ne 0 ] && exit $rc
done
done
echo "session done"
