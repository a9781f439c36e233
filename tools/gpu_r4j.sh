# GEMM / heads / conv epilogues with LDS-only barriers: tests, K-scan, same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/ab
rm -f gpurun_out/ab/summary3.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_fast.py tests/test_gpu_heads.py tests/test_gpu_conv.py tests/test_gpu_fp8.py tests/test_gpu_lstm_wide.py tests/test_gpu_parity_bench.py > gpurun_out/r4j_tests.log 2>&1 && \
GEMM_VARS=12 GEMM_EPIS=16,0 timeout -k 10 120 python -u tools/gemm_kscan.py > gpurun_out/gemm_kscan_r4j.txt 2>&1 && \
KNOB=256 CFGS="c3 c2 c5bf16 c4" bash tools/gpu_ab3.sh && mv gpurun_out/ab/summary3.txt gpurun_out/ab/summary_r4j.txt
