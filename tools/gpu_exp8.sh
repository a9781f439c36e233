# BPTT prefetch behind the poll: LSTM tests, stamps, then same-box A/B vs libmlvae_base.so
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "lstm" --timeout 120 --timeout-method thread > gpurun_out/lstm_tests.log 2>&1 && \
timeout -k 10 120 python -u tools/lstm_stamps.py 1 bwd > gpurun_out/st_bwd_pf.log 2>&1 && \
bash tools/gpu_ab.sh
