# conv slab layout + fp8 recurrence test + fp8 parity: tests, then the c4 A/B (A base lib, B new)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/ab
rm -f gpurun_out/ab/summary3.txt
timeout -k 10 500 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_lstm_wide.py tests/test_gpu_fp8.py tests/test_gpu_parity_bench.py > gpurun_out/r4q_tests.log 2>&1 && \
KNOB=0 CFGS="c4" bash tools/gpu_ab3.sh && mv gpurun_out/ab/summary3.txt gpurun_out/ab/summary_r4q_c4.txt
