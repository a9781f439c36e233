# same-box A/B, alternating: base lib (A), new lib (B), new lib + MLVAE_LSTM_DBG=$KNOB (C)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/ab
KNOB=${KNOB:-0}
for r in 1 2; do
  for c in ${CFGS:-c3 c2 c5bf16}; do
    for v in A B C; do
      if [ $v = A ]; then L=$GRAFT_REPO_ROOT/ml-vae_amd/mlvae_hip/libmlvae_base.so; K=0
      elif [ $v = B ]; then L=$GRAFT_REPO_ROOT/ml-vae_amd/mlvae_hip/libmlvae.so; K=0
      else L=$GRAFT_REPO_ROOT/ml-vae_amd/mlvae_hip/libmlvae.so; K=$KNOB; fi
      MLVAE_LIB_PATH=$L MLVAE_LSTM_DBG=$K timeout -k 10 150 python -u bench.py --config $c --no-cpu-baseline --no-extra > gpurun_out/ab/${v}_${c}_$r.json 2> gpurun_out/ab/${v}_${c}_$r.err || exit 1
      python3 -c "
import json
d=json.load(open('gpurun_out/ab/${v}_${c}_$r.json')); k=d['kernel_ms']
print('$v', '$c', $r, f\"{d['ms_per_step']:.3f} ms/step\", ' '.join(f'{n}={k[n]:.3f}' for n in ('lstm_fwd','lstm_bwd','dgrad_l1','proj_l1','conv_fwd','conv_bwd') if n in k))
" >> gpurun_out/ab/summary3.txt
    done
  done
done
