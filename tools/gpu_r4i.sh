# AS default (TPW 1), BPTT fragment batching, conv staging pipeline: tests, the tr8 probe, the GEMM
# epilogue ablation K-scan, then a same-box A/B (A base lib, B new, C new + bit 8 = equal shares)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/ab
rm -f gpurun_out/ab/summary3.txt
timeout -k 10 60 ./tools/probe_tr8 > gpurun_out/probe_tr8.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lstm_wide.py tests/test_gpu_conv.py tests/test_gpu_parity_bench.py tests/test_gpu_parity_workload.py tests/test_gpu_lstm_module.py > gpurun_out/r4i_tests.log 2>&1 && \
(for abl in 0 4 8; do MLVAE_GEMM_ABL=$abl GEMM_VARS=12 GEMM_EPIS=16 timeout -k 10 120 python -u tools/gemm_kscan.py || exit 1; done) > gpurun_out/gemm_kscan_abl.txt 2>&1 && \
KNOB=256 CFGS="c2 c5bf16 c3 c4" bash tools/gpu_ab3.sh && mv gpurun_out/ab/summary3.txt gpurun_out/ab/summary_r4i.txt
