set -u
for v in base cap8_512 cap_big; do
  lib=""; [ $v != base ] && lib="--lib tools/variants/lib_$v.so"
  timeout -k 10 150 python tools/project_ranks.py $lib --ranks 1,8 --out gpurun_out/r02i_proj_$v.json > gpurun_out/r02i_proj_$v.log 2>&1 || { echo "proj $v failed $?"; exit 1; }
  echo "== $v"; grep "^N=" gpurun_out/r02i_proj_$v.log
done
timeout -k 10 120 python tools/diag_animate.py --frames 600 --sync-every 10 > gpurun_out/r02i_diag_animate.log 2>&1; echo "diag rc $?"; tail -4 gpurun_out/r02i_diag_animate.log
