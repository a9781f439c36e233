# layer-0 input projection fused into the forward recurrence (mlvae_lstm_fwd_z): wide-kernel and
# step parity tests; steps alternating MLVAE_ZPROJ=0 (skinny projection + ex2) / 1 (fused)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lstm_wide.py tests/test_gpu_step_parity.py tests/test_gpu_parity_bench.py > gpurun_out/r4y_tests.log 2>&1 && \
rm -f gpurun_out/ab/summary_r4y.txt && \
for r in 1 2; do for c in c3 c2 c5; do for zp in 0 1; do
  MLVAE_ZPROJ=$zp timeout -k 10 150 python -u bench.py --config $c --no-cpu-baseline --no-extra > gpurun_out/ab/r4y_${zp}_${c}_$r.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/ab/r4y_${zp}_${c}_$r.json')); k=d['kernel_ms']
print('zproj=$zp', '$c', $r, f\"{d['ms_per_step']:.3f} ms/step\", ' '.join(f'{n}={v:.3f}' for n, v in sorted(k.items())))
" >> gpurun_out/ab/summary_r4y.txt
done; done; done
