# forward probes: 0 default | 1024 time-major store/load addressing (timing only) | 1 no stores
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/stamps
OUT=gpurun_out/stamps/fwd_probe3${STAMPS_TAG}.txt
run() { timeout -k 10 60 python -u tools/lstm_stamps.py "$@" >> $OUT 2>&1; }
for B in 256 64; do
  for M in 0 1024 1 0 1024; do
    echo "=== fwd B=$B mode $M" >> $OUT; run --B $B --drop 0.15 --noy --mode $M || exit 1
  done
done
