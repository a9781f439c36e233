# skinny/encoder kernel tests + step parity, then same-box A/B vs libmlvae_base.so
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_skinny.py tests/test_gpu_encoder.py tests/test_gpu_step_parity.py tests/test_gpu_dp_shards.py -x -q --timeout 120 --timeout-method thread > gpurun_out/k_tests.log 2>&1 && \
bash tools/gpu_ab.sh
