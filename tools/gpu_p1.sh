# heads P1 (split form) with two pieces in flight: heads tests + c3/c4 parity, then same-box A/B
# against the previous library (abl/libmlvae_preP1.so) at c3 and c4
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
OUT=gpurun_out/p1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_heads*.py \
  "tests/test_gpu_parity_bench.py::test_c3_headline_B256_T500_matches_oracle" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
REPS=3 bash tools/gpu_run.sh - "c3" p1ab "MLVAE_NONE=0" "MLVAE_LIB_PATH=$GRAFT_REPO_ROOT/abl/libmlvae_preP1.so"
