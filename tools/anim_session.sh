#!/bin/bash
# Motion / shadow-order checks: their GPU tests, then the shadow benches
# (dragon 1080p, happy 1080p, C5 happy 4K) with the timed push order and an
# animated dragon frame loop.
set -u
OUT=gpurun_out/${1:-anim}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "animated or headless or shadow or object_transform" > $OUT/pytest.log 2>&1 && tail -3 $OUT/pytest.log &&
timeout -k 10 300 python bench.py --steps 500 --warmup 50 --shadow --no-cpu-baseline > $OUT/shadow.log 2>&1 && tail -1 $OUT/shadow.log | cut -c1-120 &&
timeout -k 10 300 python bench.py --steps 500 --warmup 50 --shadow --scene happy --no-cpu-baseline > $OUT/happy_shadow.log 2>&1 && tail -1 $OUT/happy_shadow.log | cut -c1-120 &&
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --scene happy --width 3840 --height 2160 --shadow --no-cpu-baseline > $OUT/c5.log 2>&1 && tail -1 $OUT/c5.log | cut -c1-120 &&
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --animate "R+W.Q.T.W" --no-cpu-baseline > $OUT/anim.log 2>&1 && tail -1 $OUT/anim.log | cut -c1-120
