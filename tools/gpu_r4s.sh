# GEMM tile-order group size (MLVAE_GEMM_GROUP_M) K-scan + c3 step A/B; conv prologue (new
# library) tests + c4
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/ab
(for gm in 4 1 2 8 16; do MLVAE_GEMM_GROUP_M=$gm GEMM_VARS=12 GEMM_EPIS=16 timeout -k 10 120 python -u tools/gemm_kscan.py | sed "s/^/gm=$gm /" || exit 1; done) > gpurun_out/gemm_kscan_gm.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv.py > gpurun_out/r4s_tests.log 2>&1 && \
rm -f gpurun_out/ab/summary3.txt && KNOB=0 CFGS="c4" bash tools/gpu_ab3.sh && mv gpurun_out/ab/summary3.txt gpurun_out/ab/summary_r4s_c4.txt
