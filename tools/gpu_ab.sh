# same-box A/B of two builds: libmlvae_base.so (A) vs libmlvae.so (B), alternating bench runs
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
for r in 1 2; do
  MLVAE_LIB_PATH=$GRAFT_REPO_ROOT/ml-vae_amd/mlvae_hip/libmlvae_base.so timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/ab_A$r.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/ab_B$r.log 2>&1 || exit 1
done
