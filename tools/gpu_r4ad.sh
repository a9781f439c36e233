# layer-0 dZ + dW_ih_l0 from one pass over dG (mlvae_skinny_dzw) vs the NT + TN pair (MLVAE_DZW=0):
# skinny / step parity tests, c3 and c2 alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_skinny.py tests/test_gpu_step_parity.py tests/test_gpu_parity_bench.py tests/test_gpu_parity_workload.py > gpurun_out/r4ad_tests.log 2>&1 && \
rm -f gpurun_out/ab/summary_r4ad.txt && \
for r in 1 2; do for c in c3 c2; do for v in 0 1; do
  MLVAE_DZW=$v timeout -k 10 150 python -u bench.py --config $c --no-cpu-baseline --no-extra > gpurun_out/ab/r4ad_${v}_${c}_$r.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/ab/r4ad_${v}_${c}_$r.json')); k=d['kernel_ms']
print('dzw=$v', '$c', $r, f\"{d['ms_per_step']:.3f} ms/step\", ' '.join(f'{n}={v:.3f}' for n, v in sorted(k.items())))
" >> gpurun_out/ab/summary_r4ad.txt
done; done; done && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dzw -o run -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/prof_dzw.log 2>&1
