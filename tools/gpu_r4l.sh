# fp8 wgrad debug probe; persistent GEMM (VAR 14): tests, K-scan, same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/ab
rm -f gpurun_out/ab/summary3.txt
timeout -k 10 200 python -u tools/dbg_fp8w.py > gpurun_out/dbg_fp8w.txt 2>&1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_fast.py tests/test_gpu_heads.py > gpurun_out/r4l_tests.log 2>&1 && \
GEMM_VARS=0,12 GEMM_EPIS=16,0 timeout -k 10 200 python -u tools/gemm_kscan.py > gpurun_out/gemm_kscan_r4l.txt 2>&1 && \
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity_bench.py tests/test_gpu_parity_workload.py -k "not c5_fp8_second" > gpurun_out/r4l_parity.log 2>&1 && \
KNOB=0 CFGS="c3 c2 c5bf16" bash tools/gpu_ab3.sh && mv gpurun_out/ab/summary3.txt gpurun_out/ab/summary_r4l.txt
