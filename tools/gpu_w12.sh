# The 12-wave TPW-1 forward as the default: parity through the step at every TPW-1 shape, then
# same-box A/B against the 8-wave form (bit 11) at the shards it runs (c5 shard, c4, c3h).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
OUT=gpurun_out/w12
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_lstm_wide.py tests/test_gpu_parity_bench.py tests/test_gpu_parity_workload.py \
  tests/test_gpu_step_parity.py tests/test_gpu_trajectory.py \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
REPS=2 bash tools/gpu_run.sh - "c5bf16 c4 c3h" w12ab "MLVAE_LSTM_DBG=0" "MLVAE_LSTM_DBG=2048"
