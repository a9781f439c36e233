# io waves behind the poll: LSTM tests + stamps fwd/bwd + bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "lstm" --timeout 120 --timeout-method thread > gpurun_out/lstm_tests.log 2>&1 && \
timeout -k 10 120 python -u tools/lstm_stamps.py 1 > gpurun_out/st_fwd_io.log 2>&1 && \
timeout -k 10 120 python -u tools/lstm_stamps.py 1 bwd > gpurun_out/st_bwd_io.log 2>&1 && \
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_io.log 2>&1
