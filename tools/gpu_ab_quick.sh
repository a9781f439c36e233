# same-box A/B, alternating: libmlvae_base.so (A) vs libmlvae.so (B), bench --no-extra on the
# configs given (default c3 c2); summary lines into gpurun_out/ab/summary.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/ab
CFGS=${*:-c3 c2}
for r in 1 2; do
  for c in $CFGS; do
    MLVAE_LIB_PATH=$GRAFT_REPO_ROOT/ml-vae_amd/mlvae_hip/libmlvae_base.so timeout -k 10 150 python -u bench.py --config $c --no-cpu-baseline --no-extra > gpurun_out/ab/A_${c}_$r.json 2> gpurun_out/ab/A_${c}_$r.err || exit 1
    timeout -k 10 150 python -u bench.py --config $c --no-cpu-baseline --no-extra > gpurun_out/ab/B_${c}_$r.json 2> gpurun_out/ab/B_${c}_$r.err || exit 1
    python3 -c "
import json,sys
for t in 'AB':
    d=json.load(open(f'gpurun_out/ab/{t}_${c}_$r.json'))
    k=d['kernel_ms']
    print(t, '${c}', $r, f\"{d['ms_per_step']:.3f} ms/step\", ' '.join(f'{n}={k[n]:.3f}' for n in ('lstm_fwd','lstm_bwd','dgrad_l1','proj_l1') if n in k))
" >> gpurun_out/ab/summary.txt
  done
done
