# recurrence timing: default vs no in-loop prefetch (dbg bit 11) vs no stores (bit 0)
set -o pipefail
cd $GRAFT_REPO_ROOT
for m in 0 2048 2049; do
  LSTM_DBG_MODE=$m timeout -k 10 120 python -u tools/lstm_stamps.py 1 > gpurun_out/st_fwd_$m.log 2>&1 || exit 1
  LSTM_DBG_MODE=$m timeout -k 10 120 python -u tools/lstm_stamps.py 1 bwd > gpurun_out/st_bwd_$m.log 2>&1 || exit 1
done
