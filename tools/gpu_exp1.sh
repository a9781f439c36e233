# A/B of recurrence switches (lstm.hip diagnostics mode bits): isolated stamps + training bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
out=gpurun_out/exp1; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $out/pytest_kernels.log 2>&1 || exit 1
for m in 0 2 16 18; do
  LSTM_DBG_MODE=$m timeout -k 10 60 python -u tools/lstm_stamps.py 1 > $out/fwd_$m.log 2>&1 || exit 1
done
for m in 0 2 16; do
  LSTM_DBG_MODE=$m timeout -k 10 60 python -u tools/lstm_stamps.py 1 bwd > $out/bwd_$m.log 2>&1 || exit 1
done
for m in 0 8 16 2 10; do
  MLVAE_LSTM_MODE=$m timeout -k 10 120 python -u bench.py --no-cpu-baseline > $out/bench_$m.log 2>&1 || exit 1
done
