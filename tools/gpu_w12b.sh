# The 12-wave TPW-1 BPTT: parity (fp64 loop, whole steps), stamps, same-box A/B against 8 waves (bit 5)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
OUT=gpurun_out/w12b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_lstm_wide.py ${W12B_TESTS:-} > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
DL=$GRAFT_REPO_ROOT/ml-vae_amd/mlvae_hip/libmlvae_diag.so
for m in 0 32; do
  echo "=== bwd B=32 mode $m" >> $OUT/stamps.txt
  MLVAE_LIB_PATH=$DL timeout -k 10 60 python -u tools/lstm_stamps.py --B 32 --bwd --mode $m >> $OUT/stamps.txt 2>&1 || exit 1
done
REPS=2 bash tools/gpu_run.sh - "${W12B_CFGS:-c2 c5bf16}" w12bab "MLVAE_LSTM_DBG=0" "MLVAE_LSTM_DBG=32"
