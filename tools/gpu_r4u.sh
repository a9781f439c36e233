# conv persistent grid (MLVAE_CONV_MULT 1 / 2 / 3) at c4; GEMM group 8 default: gemm tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gemm_fast.py tests/test_gpu_conv.py > gpurun_out/r4u_tests.log 2>&1 && \
rm -f gpurun_out/ab/summary_cm.txt && \
for r in 1 2; do for m in 2 1 3; do
  MLVAE_CONV_MULT=$m timeout -k 10 150 python -u bench.py --config c4 --no-cpu-baseline --no-extra > gpurun_out/ab/cm_${m}_$r.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/ab/cm_${m}_$r.json')); k=d['kernel_ms']
print('conv_mult=$m', $r, f\"{d['ms_per_step']:.3f} ms/step\", ' '.join(f'{n}={v:.3f}' for n, v in sorted(k.items()) if n.startswith('conv')))
" >> gpurun_out/ab/summary_cm.txt
done; done
