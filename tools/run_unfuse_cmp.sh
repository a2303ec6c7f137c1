set -u
cd "${GRAFT_REPO_ROOT}"
bash tools/gpu_round.sh || exit $?
for uf in 1 4; do
  MIMI_HIP_UNFUSE_FROM=$uf timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 > gpurun_out/bench_uf$uf.log 2>&1 || exit $?
done
echo done
