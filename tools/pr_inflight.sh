set -u
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/r02s2_pr
for L in 2 3 4; do
  timeout -k 10 200 python tools/project_ranks.py --inflight $L --ranks 1,2,4,8 --frames 400 --out gpurun_out/r02s2_pr/inflight$L.json > gpurun_out/r02s2_pr/inflight$L.log 2>&1 || exit $?
  tail -6 gpurun_out/r02s2_pr/inflight$L.log
done
