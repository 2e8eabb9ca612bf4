#!/bin/bash
# Per-slot order-upload waits: GPU tests, then the moving bench three times and C4 once.
set -u
TAG=${1:-s3m}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "== pytest exit $rc"; tail -1 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 500 --warmup 20 --animate R+W.Q.T.W --no-cpu-baseline > "$OUT/anim_r$rep.log" 2>&1
  rc=$?
  echo "== anim rep $rep exit $rc"; grep '^{' "$OUT/anim_r$rep.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], r['kernel_ms_avg'], r['kernel_ms_avg_timed'], d['host']['us_per_frame'], d['frame_check']['matches_oracle'], d['device_err'])"
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 200 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline > "$OUT/c4.log" 2>&1
rc=$?; echo "== c4 exit $rc"; grep '^{' "$OUT/c4.log" | cut -c1-200
echo "session done"
