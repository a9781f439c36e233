# per-phase stamps (LDS-buffered, steps 64..95) of the wide recurrences, fwd and bwd, B=256 / 32;
# extra args (e.g. debug-mode bits) go to every run: bash tools/gpu_stamps.sh [--mode N]
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/stamps
OUT=gpurun_out/stamps/stamps${STAMPS_TAG}.txt
run() { timeout -k 10 60 python -u tools/lstm_stamps.py "$@" >> $OUT 2>&1; }
for B in 256 32; do
  echo "=== fwd B=$B $*" >> $OUT; run --B $B --drop 0.15 --noy "$@" || exit 1
  echo "=== bwd B=$B $*" >> $OUT; run --B $B --bwd "$@" || exit 1
done
