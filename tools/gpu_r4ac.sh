# full-chip step tail: dW_hh_l0 on the side stream beside dZ / encoder backward / dW_ih_l0
# (MLVAE_TAIL_OVERLAP=1) vs serialised (0): step parity tests, c3 alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_step_parity.py tests/test_gpu_parity_bench.py tests/test_gpu_parity_workload.py > gpurun_out/r4ac_tests.log 2>&1 && \
rm -f gpurun_out/ab/summary_r4ac.txt && \
for r in 1 2 3; do for v in 0 1; do
  MLVAE_TAIL_OVERLAP=$v timeout -k 10 150 python -u bench.py --config c3 --no-cpu-baseline --no-extra > gpurun_out/ab/r4ac_${v}_$r.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/ab/r4ac_${v}_$r.json')); k=d['kernel_ms']
print('tail_overlap=$v', $r, f\"{d['ms_per_step']:.3f} ms/step\", ' '.join(f'{n}={v:.3f}' for n, v in sorted(k.items())))
" >> gpurun_out/ab/summary_r4ac.txt
done; done
