# GEMM main loop: a variant (TVAR, default VAR 16) against the default (VAR 12): the c3 shapes in one
# process, the 256^2 tests under the variant, then same-box A/B in the step
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/g16
GEMM_FRAMES=128000 GEMM_VARS=${GEMM_VARS:-12,16} GEMM_ONLY="${GEMM_ONLY:-}" timeout -k 10 300 python -u tools/gemm_bench.py > gpurun_out/g16/ab.txt 2>&1 || exit 1
cat gpurun_out/g16/ab.txt
MLVAE_GEMM_VAR=${TVAR:-16} timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gemm_fast.py > gpurun_out/g16/pytest.log 2>&1; tail -2 gpurun_out/g16/pytest.log
REPS=2 bash tools/gpu_run.sh - "${STEP_CFGS:-c3}" gvar "MLVAE_NONE=0" "MLVAE_GEMM_VAR=${TVAR:-16}"
