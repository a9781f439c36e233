# forward-recurrence probes: per-phase stamps at B=256 / 32 with the io traffic switched off
# piece by piece (debug-mode bits: 1 = no saved-activation stores, 8192 = no gx loads)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/stamps
OUT=gpurun_out/stamps/fwd_probe${STAMPS_TAG}.txt
run() { timeout -k 10 60 python -u tools/lstm_stamps.py "$@" >> $OUT 2>&1; }
for B in 256 32; do
  for M in 0 1 8192 8193; do
    echo "=== fwd B=$B mode $M" >> $OUT; run --B $B --drop 0.15 --noy --mode $M || exit 1
  done
done
