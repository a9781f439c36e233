# 16-byte (8-column) 16-bit C epilogue stores vs the 4-column ones (MLVAE_GEMM_ABL=64): GEMM tests,
# K-scan (fp16 C), c3 / c2 steps alternating on the same box
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gemm_fast.py tests/test_gpu_fp8.py > gpurun_out/r4v_tests.log 2>&1 && \
rm -f gpurun_out/ab/kscan_w8.txt && \
for a in 0 64; do MLVAE_GEMM_ABL=$a GEMM_VARS=12 GEMM_EPIS=16 timeout -k 10 200 python -u tools/gemm_kscan.py >> gpurun_out/ab/kscan_w8.txt 2>&1 || exit 1; done && \
rm -f gpurun_out/ab/summary_w8.txt && \
for r in 1 2; do for c in c3 c2; do for a in 64 0; do
  MLVAE_GEMM_ABL=$a timeout -k 10 150 python -u bench.py --config $c --no-cpu-baseline --no-extra > gpurun_out/ab/w8_${c}_${a}_$r.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/ab/w8_${c}_${a}_$r.json')); k=d['kernel_ms']
print('$c abl=$a', $r, f\"{d['ms_per_step']:.3f} ms/step\", ' '.join(f'{n}={v:.3f}' for n, v in sorted(k.items())))
" >> gpurun_out/ab/summary_w8.txt
done; done; done
