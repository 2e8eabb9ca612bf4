#!/bin/bash
set -u
OUT=gpurun_out/r02b; mkdir -p $OUT
timeout -k 10 60 tools/ubench_pk > $OUT/ubench.log 2>&1; echo "ubench rc $?"; cat $OUT/ubench.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "flat" > $OUT/pytest_flat.log 2>&1; rc=$?; echo "pytest rc $rc"; tail -3 $OUT/pytest_flat.log
[ $rc -le 1 ] || exit $rc
for v in 0 1 2; do
  timeout -k 10 300 python bench.py --scene rabbit_70k --width 960 --height 540 --mode 1 --steps 30 --warmup 3 --flat $v --no-cpu-baseline > $OUT/bench_flat_v$v.log 2>&1 || exit $?
done
python tools/bench_summary.py $OUT/bench_flat_v*.log
