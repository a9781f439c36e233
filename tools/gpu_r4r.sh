# the committed state vs the previous commit's library (A): c3 / c2 / c5bf16; C = the forward's
# s_sleep 1 retry back-off at full chip (debug bit 30)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/ab
rm -f gpurun_out/ab/summary3.txt
KNOB=1073741824 CFGS="c3 c2 c5bf16" bash tools/gpu_ab3.sh && mv gpurun_out/ab/summary3.txt gpurun_out/ab/summary_r4r.txt
[ -f gpurun_out/ab/summary_r4r.txt ] || exit 1
rm -f gpurun_out/ab/summary_wgm.txt
for r in 1 2; do for m in 1 2; do
  MLVAE_CONV_WG_MULT=$m timeout -k 10 150 python -u bench.py --config c4 --no-cpu-baseline --no-extra > gpurun_out/ab/wgm_${m}_$r.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/ab/wgm_${m}_$r.json')); k=d['kernel_ms']
print('wg_mult=$m', $r, f\"{d['ms_per_step']:.3f} ms/step\", ' '.join(f'{n}={v:.3f}' for n, v in sorted(k.items()) if n.startswith('conv')))
" >> gpurun_out/ab/summary_wgm.txt
done; done
