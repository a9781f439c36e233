# conv staging pipeline + asymmetric tile split (TPW 1, debug bit 8): correctness, then same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/ab
rm -f gpurun_out/ab/summary3.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_lstm_wide.py > gpurun_out/r4h_tests.log 2>&1 && \
MLVAE_LSTM_DBG=256 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lstm_wide.py > gpurun_out/r4h_tests_as.log 2>&1 && \
KNOB=256 CFGS="c2 c5bf16 c3 c4" bash tools/gpu_ab3.sh && mv gpurun_out/ab/summary3.txt gpurun_out/ab/summary_as.txt && \
timeout -k 10 240 python -u tools/gemm_kscan.py > gpurun_out/gemm_kscan.txt 2>&1
