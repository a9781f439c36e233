set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/stamps gpurun_out/knob
O=gpurun_out/stamps/handoff.txt
for args in "--B 256" "--B 256 --mode 1" "--B 64" "--B 64 --mode 1"; do
  timeout -k 10 60 python -u tools/lstm_handoff.py $args >> $O 2>&1 || exit 1
done
O=gpurun_out/stamps/bwd_probe.txt
for B in 256 64; do
  for M in 0 131072 524288 655360 0; do
    echo "=== bwd B=$B mode $M" >> $O
    timeout -k 10 60 python -u tools/lstm_stamps.py --B $B --bwd --mode $M >> $O 2>&1 || exit 1
  done
done
for r in 1 2; do
  for v in 0 131072 524288 655360; do
    MLVAE_LSTM_DBG=$v timeout -k 10 150 python -u bench.py --config c3 --no-cpu-baseline --no-extra > gpurun_out/knob/c3_${v}_${r}.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/knob/c3_${v}_${r}.json')); k=d['kernel_ms']
print('c3 dbg $v run $r', f\"{d['ms_per_step']:.3f} ms/step\", f\"fwd {k['lstm_fwd']:.3f} bwd {k['lstm_bwd']:.3f}\")" >> gpurun_out/knob/summary.txt
  done
done
