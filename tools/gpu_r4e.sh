set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/stamps
O=gpurun_out/stamps/io_phases.txt
for B in 256 64; do
  for M in 16 17; do
    echo "=== fwd B=$B mode $M" >> $O
    timeout -k 10 60 python -u tools/lstm_stamps.py --B $B --drop 0.15 --noy --mode $M >> $O 2>&1 || exit 1
  done
done
