set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_lstm_wide.py tests/test_gpu_trajectory.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_wt.log 2>&1 && \
bash tools/gpu_fwd_probe3.sh && \
bash tools/gpu_ab_quick.sh c3 c2 c5bf16 && \
bash tools/gpu_check.sh
