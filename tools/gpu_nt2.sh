# The 32-utterance forward (NT = 2) in 12 waves: parity against the fp64 loop and through the
# step, stamps of the forms (diagnostics build; bit 9 = the TPW-2 form, bit 11 = the other
# 12-wave choice), same-box A/B in the step.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
OUT=gpurun_out/nt2
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_lstm_wide.py "tests/test_gpu_parity_bench.py::test_c3_headline_B256_T500_matches_oracle" \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
DL=$GRAFT_REPO_ROOT/ml-vae_amd/mlvae_hip/libmlvae_diag.so
for m in 0 512 2048; do
  echo "=== fwd B=256 mode $m" >> $OUT/stamps.txt
  MLVAE_LIB_PATH=$DL timeout -k 10 60 python -u tools/lstm_stamps.py --B 256 --drop 0.15 --noy --mode $m >> $OUT/stamps.txt 2>&1 || exit 1
done
for m in 0 2048; do
  echo "=== fwd B=32 mode $m" >> $OUT/stamps.txt
  MLVAE_LIB_PATH=$DL timeout -k 10 60 python -u tools/lstm_stamps.py --B 32 --drop 0.15 --noy --mode $m >> $OUT/stamps.txt 2>&1 || exit 1
done
REPS=2 bash tools/gpu_run.sh - "c3" nt2ab "MLVAE_LSTM_DBG=0" "MLVAE_LSTM_DBG=512"
REPS=2 bash tools/gpu_run.sh - "c2" nt2ab_c2 "MLVAE_LSTM_DBG=0" "MLVAE_LSTM_DBG=2048"
