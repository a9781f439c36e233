# GEMM tile order: groups of G M-panels (MLVAE_GEMM_GROUP_M) on the c3 projection / dgrad shapes,
# then the c3 step for the default (8) against the best alternative
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
OUT=gpurun_out/grpm
mkdir -p $OUT
for G in 8 2 4 16 8 2 4 16; do
  echo "group_m=$G" >> $OUT/bench.txt
  MLVAE_GEMM_GROUP_M=$G GEMM_FRAMES=128000 GEMM_MODES=1 GEMM_ONLY=dgrad timeout -k 10 120 python -u tools/gemm_bench.py >> $OUT/bench.txt 2>&1 || exit 1
  MLVAE_GEMM_GROUP_M=$G GEMM_FRAMES=128000 GEMM_MODES=1 GEMM_ONLY="fwd proj" timeout -k 10 120 python -u tools/gemm_bench.py >> $OUT/bench.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $OUT/bench.txt
REPS=2 bash tools/gpu_run.sh - "c3" grpmab "MLVAE_GEMM_GROUP_M=8" "MLVAE_GEMM_GROUP_M=${GBEST:-2}" "MLVAE_GEMM_GROUP_M=4"
