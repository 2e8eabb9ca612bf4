mkdir -p gpurun_out/r01h
for lib in cpp_cuda_raytracer_dev_amd/librt_mi355x.so tools/variants/lib_c16_448_c32_448.so tools/variants/lib_c16_640_c32_640.so; do
  for r in 16 32; do
    timeout -k 10 200 python tools/bench_variant.py $lib --steps 300 --warmup 30 --no-cpu-baseline --rays $r --items 2 > gpurun_out/r01h/b.log 2>&1 || exit 3
    echo "$lib r$r: $(grep -o '"value": [0-9.]*' gpurun_out/r01h/b.log) $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/r01h/b.log)"
  done
done
timeout -k 10 200 python tools/diag_waves.py dragon 1920 1080 3 16 2 2 > gpurun_out/r01h/diag16.log 2>&1 && tail -1 gpurun_out/r01h/diag16.log
