# encoder backward with the next tile's inputs prefetched: encoder / step parity tests, then
# c3 and c2 alternating A = libmlvae_base.so (before), B = new
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_encoder.py tests/test_gpu_step_parity.py tests/test_gpu_parity_bench.py > gpurun_out/r4ae_tests.log 2>&1 && \
rm -f gpurun_out/ab/summary_r4ae.txt && \
for r in 1 2; do for c in c3 c2; do for v in A B; do
  if [ $v = A ]; then L=$GRAFT_REPO_ROOT/ml-vae_amd/mlvae_hip/libmlvae_base.so; else L=$GRAFT_REPO_ROOT/ml-vae_amd/mlvae_hip/libmlvae.so; fi
  MLVAE_LIB_PATH=$L timeout -k 10 150 python -u bench.py --config $c --no-cpu-baseline --no-extra > gpurun_out/ab/r4ae_${v}_${c}_$r.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/ab/r4ae_${v}_${c}_$r.json')); k=d['kernel_ms']
print('$v', '$c', $r, f\"{d['ms_per_step']:.3f} ms/step\", ' '.join(f'{n}={v:.3f}' for n, v in sorted(k.items()) if n.startswith('enc')))
" >> gpurun_out/ab/summary_r4ae.txt
done; done; done
