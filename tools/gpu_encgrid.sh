# encoder forward workgroup cap (MLVAE_ENC_GRID, A/B build), c3 and c2 alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_encoder.py > gpurun_out/encg_pytest.log 2>&1 || { tail -20 gpurun_out/encg_pytest.log; exit 1; }
MLVAE_ENC_GRID=1024 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_encoder.py >> gpurun_out/encg_pytest.log 2>&1 || { tail -20 gpurun_out/encg_pytest.log; exit 1; }
grep passed gpurun_out/encg_pytest.log
REPS=2 bash tools/gpu_run.sh - "c3 c2" encg "MLVAE_ENC_GRID=256" "MLVAE_ENC_GRID=512" "MLVAE_ENC_GRID=1024"
