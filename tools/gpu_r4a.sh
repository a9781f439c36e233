set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/stamps
MLVAE_LIB_PATH=$GRAFT_REPO_ROOT/ml-vae_amd/mlvae_hip/libmlvae_base.so timeout -k 10 90 python -u tools/epi_bench.py > gpurun_out/stamps/epi_bench_base.txt 2>&1 && \
bash tools/gpu_fwd_probe.sh && \
bash tools/gpu_ab_quick.sh c3 c2 && \
bash tools/gpu_check.sh
