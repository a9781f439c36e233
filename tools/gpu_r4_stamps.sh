# phase stamps of the final round-4 recurrences (diagnostics for the step-latency work):
# forward and BPTT at B = 256 (TPW 2) and B = 32 (TPW 1, asymmetric forward)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out
{ timeout -k 10 120 python -u tools/lstm_stamps.py --B 256 && \
  timeout -k 10 120 python -u tools/lstm_stamps.py --B 256 --bwd && \
  timeout -k 10 120 python -u tools/lstm_stamps.py --B 32 && \
  timeout -k 10 120 python -u tools/lstm_stamps.py --B 32 --bwd; } > gpurun_out/r04_lstm_stamps.txt 2>&1
