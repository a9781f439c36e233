set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_lstm_wide.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_wide.log 2>&1 && \
bash tools/gpu_fwd_probe2.sh && \
timeout -k 10 500 python -u -m pytest tests/test_gpu_trajectory.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_traj.log 2>&1
