set -u
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > gpurun_out/r02k_pytest.log 2>&1; rc=$?; echo "pytest rc $rc"; tail -2 gpurun_out/r02k_pytest.log; [ $rc -le 1 ] || exit $rc
for v in new dblpred; do
  lib=""; [ $v != new ] && lib="--lib tools/variants/lib_$v.so"
  timeout -k 10 150 python tools/project_ranks.py $lib --ranks 1,8 --out gpurun_out/r02k_proj_$v.json > gpurun_out/r02k_proj_$v.log 2>&1 || { echo "proj $v failed"; exit 1; }
  echo "== $v"; grep "^N=" gpurun_out/r02k_proj_$v.log
done
timeout -k 10 100 python tools/bench_variant.py tools/variants/lib_dblpred.so --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/r02k_c4_dbl.log 2>&1
timeout -k 10 100 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/r02k_c4_new.log 2>&1
timeout -k 10 100 python bench.py --steps 300 --warmup 30 --view fill --no-cpu-baseline > gpurun_out/r02k_fill_new.log 2>&1
timeout -k 10 100 python tools/bench_variant.py tools/variants/lib_dblpred.so --steps 300 --warmup 30 --view fill --no-cpu-baseline > gpurun_out/r02k_fill_dbl.log 2>&1
python tools/bench_summary.py gpurun_out/r02k_c4_*.log gpurun_out/r02k_fill_*.log
