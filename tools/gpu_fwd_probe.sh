# forward-recurrence probes: per-phase stamps at B=256 / 32 with the io traffic switched off
# piece by piece (debug-mode bits: 1 = no saved-activation stores, 8192 = no gx loads,
# 8388608 (bit 23) = stamp the publish stores' ack, 67108864 (bit 26) = pollers' MFMAs first,
# 131072 (bit 17) = io stores behind every wave's publish, 524288 (bit 19) = io stores from
# registers right after the barrier)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/stamps
OUT=gpurun_out/stamps/fwd_probe${STAMPS_TAG}.txt
run() { timeout -k 10 60 python -u tools/lstm_stamps.py "$@" >> $OUT 2>&1; }
timeout -k 10 90 python -u tools/epi_bench.py > gpurun_out/stamps/epi_bench.txt 2>&1 || exit 1
for B in 256 32; do
  for M in 0 1 8192 8193 8388608 8388609 67108864 131072 524288 8912896; do
    echo "=== fwd B=$B mode $M" >> $OUT; run --B $B --drop 0.15 --noy --mode $M || exit 1
  done
  for M in 0 1 524288; do   # the top layer's form: no dropout(h) output, no keep bits
    echo "=== fwd B=$B nodrop mode $M" >> $OUT; run --B $B --drop 0 --noy --mode $M || exit 1
  done
done
