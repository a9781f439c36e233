# forward-recurrence stamps under timing-only debug modes (diagnostics build): which part of the
# io waves' work holds the step barrier.  bash tools/gpu_fwd_modes.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 MLVAE_LIB_PATH=$GRAFT_REPO_ROOT/ml-vae_amd/mlvae_hip/libmlvae_diag.so
mkdir -p gpurun_out/stamps
OUT=gpurun_out/stamps/fwd_modes.txt
for m in ${MODES:-0 16}; do
  echo "=== fwd B=256 mode $m" >> $OUT
  timeout -k 10 60 python -u tools/lstm_stamps.py --B 256 --drop 0.15 --noy --mode $m >> $OUT 2>&1 || exit 1
done
