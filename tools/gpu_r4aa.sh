# fused Conv1d backward (mlvae_conv1d_bwd2) vs dgrad + wgrad (MLVAE_CONV_BWD2=0): conv tests
# (incl. bit-identity with the two kernels and the c4 step vs the oracle), c4 steps alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py > gpurun_out/r4aa_tests.log 2>&1 && \
rm -f gpurun_out/ab/summary_r4aa.txt && \
for r in 1 2; do for v in 0 1; do
  MLVAE_CONV_BWD2=$v timeout -k 10 200 python -u bench.py --config c4 --no-cpu-baseline --no-extra > gpurun_out/ab/r4aa_${v}_$r.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/ab/r4aa_${v}_$r.json')); k=d['kernel_ms']
print('conv_bwd2=$v', $r, f\"{d['ms_per_step']:.3f} ms/step\", ' '.join(f'{n}={v:.4f}' for n, v in sorted(k.items()) if n.startswith('conv')))
" >> gpurun_out/ab/summary_r4aa.txt
done; done && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4c -o run -- python3 -u bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/prof_c4c.log 2>&1
