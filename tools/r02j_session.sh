set -u
run() { tag=$1; shift; timeout -k 10 150 python tools/project_ranks.py --ranks 1,8 --out gpurun_out/r02j_$tag.json "$@" > gpurun_out/r02j_$tag.log 2>&1 || { echo "proj $tag failed $?"; exit 1; }; echo "== $tag"; grep "^N=" gpurun_out/r02j_$tag.log; }
run cap512_i2
run cap512_i1 --items 1
run cap640_i2 --lib tools/variants/lib_cap8_640.so
run cap512_r8 --rays 8
run cap512_r8_i1 --rays 8 --items 1
timeout -k 10 100 python bench.py --width 960 --height 540 --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/r02j_c3.log 2>&1; python tools/bench_summary.py gpurun_out/r02j_c3.log
