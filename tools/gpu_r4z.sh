# (1) ping-pong main-loop ablations (VAR 13: bit 1 no MFMAs, bit 2 no staging; bit 8 no epilogue);
# (2) c4 with the whole Conv1d backward in the timed region; (3) c5 fp8 vs bf16, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_parity_bench.py tests/test_gpu_gemm_fast.py > gpurun_out/r4z_tests.log 2>&1 && \
rm -f gpurun_out/ab/kscan_abl13.txt && \
for a in 8 9 10 11; do MLVAE_GEMM_ABL=$a GEMM_VARS=13 GEMM_EPIS=16 timeout -k 10 200 python -u tools/gemm_kscan.py >> gpurun_out/ab/kscan_abl13.txt 2>&1 || exit 1; done && \
rm -f gpurun_out/ab/summary_r4z.txt && \
for r in 1 2; do for c in c4 c5 c5bf16; do
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --no-extra > gpurun_out/ab/r4z_${c}_$r.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/ab/r4z_${c}_$r.json')); k=d['kernel_ms']
print('$c', $r, f\"{d['ms_per_step']:.3f} ms/step\", ' '.join(f'{n}={v:.3f}' for n, v in sorted(k.items())), json.dumps(d.get('roofline')))
" >> gpurun_out/ab/summary_r4z.txt
done; done
