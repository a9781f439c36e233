# forward-recurrence variant probes (stamps + launch time), B = 256 / 64 / 32:
#   0 default | 512 XL whole-line exchange | 536870912 QF quarter flags (io stores after the
#   polls) | 536871424 QF + XL | 524288 IOV 2 | 524800 IOV 2 + XL | 513 XL without stores
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/stamps
OUT=gpurun_out/stamps/fwd_probe2${STAMPS_TAG}.txt
run() { timeout -k 10 60 python -u tools/lstm_stamps.py "$@" >> $OUT 2>&1; }
for B in 256 64 32; do
  for M in 0 512 536870912 536871424 524288 524800 513 0; do
    echo "=== fwd B=$B mode $M" >> $OUT; run --B $B --drop 0.15 --noy --mode $M || exit 1
  done
done
