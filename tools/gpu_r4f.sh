set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/stamps
timeout -k 10 300 python -u -m pytest tests/test_gpu_lstm_wide.py tests/test_gpu_parity_bench.py -x -q -s --timeout 200 --timeout-method thread > gpurun_out/pytest_r4f.log 2>&1 && \
timeout -k 10 60 python -u tools/lstm_handoff.py --B 256 > gpurun_out/stamps/handoff2.txt 2>&1 && \
timeout -k 10 60 python -u tools/lstm_handoff.py --B 256 --mode 131072 >> gpurun_out/stamps/handoff2.txt 2>&1 && \
timeout -k 10 60 python -u tools/lstm_handoff.py --B 64 --mode 131072 >> gpurun_out/stamps/handoff2.txt 2>&1 && \
KNOB=131072 bash tools/gpu_ab3.sh
