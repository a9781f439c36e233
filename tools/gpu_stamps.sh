set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/lstm_stamps.py 1 > gpurun_out/stamps_fwd.log 2>&1 && \
LSTM_DBG_MODE=1 timeout -k 10 120 python -u tools/lstm_stamps.py 1 > gpurun_out/stamps_fwd_nostore.log 2>&1 && \
timeout -k 10 120 python -u tools/lstm_stamps.py 1 bwd > gpurun_out/stamps_bwd.log 2>&1 && \
LSTM_DBG_MODE=1 timeout -k 10 120 python -u tools/lstm_stamps.py 1 bwd > gpurun_out/stamps_bwd_nostore.log 2>&1
