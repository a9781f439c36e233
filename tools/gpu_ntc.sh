# non-temporal 16-bit C stores (MLVAE_GEMM_ABL=128: the projection's fp16 gx, the dgrad's bf16 dY)
# against plain stores, same box alternating (c3, c2)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
GEMM_FRAMES=128000 GEMM_MODES=1 GEMM_ONLY="fwd proj" timeout -k 10 120 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu
MLVAE_GEMM_ABL=128 GEMM_FRAMES=128000 GEMM_MODES=1 GEMM_ONLY="fwd proj" timeout -k 10 120 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu
REPS=3 bash tools/gpu_run.sh - "c3 c2" ntc "MLVAE_NONE=0" "MLVAE_GEMM_ABL=128"
