# A/B of the 256² GEMM tile order (MLVAE_GEMM_GROUP_M) + the bucketed all-reduce ordering test
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 200 python -u -m pytest tests/test_gpu_dp_shards.py -x -v --timeout 120 --timeout-method thread > gpurun_out/dp.log 2>&1 && \
for g in 0 4 8; do
  MLVAE_GEMM_GROUP_M=$g timeout -k 10 200 python -u tools/gemm_bench.py > gpurun_out/gemm_g$g.log 2>&1 || exit 1
done && \
for g in 0 4; do
  MLVAE_GEMM_GROUP_M=$g timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_g$g.log 2>&1 || exit 1
done
