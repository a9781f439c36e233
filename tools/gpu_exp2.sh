# recurrence: delayed first poll sweep (mode bits 5-10), isolated stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
out=gpurun_out/exp2; mkdir -p $out
for d in 0 4 8 12 16 24; do
  m=$((d * 32))
  LSTM_DBG_MODE=$m timeout -k 10 60 python -u tools/lstm_stamps.py 1 > $out/fwd_$d.log 2>&1 || exit 1
  LSTM_DBG_MODE=$m timeout -k 10 60 python -u tools/lstm_stamps.py 1 bwd > $out/bwd_$d.log 2>&1 || exit 1
done
