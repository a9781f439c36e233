# GEMM epilogue: nt stores A/B (MLVAE_GEMM_ABL=32) in the K-scan; c3 stamps of the recurrences
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
(for abl in 0 32; do MLVAE_GEMM_ABL=$abl GEMM_VARS=12 GEMM_EPIS=16,0 timeout -k 10 120 python -u tools/gemm_kscan.py || exit 1; done) > gpurun_out/gemm_kscan_r4o.txt 2>&1 && \
rm -f gpurun_out/ab/summary_abl.txt && \
for r in 1 2; do for abl in 0 32; do
  MLVAE_GEMM_ABL=$abl timeout -k 10 150 python -u bench.py --config c3 --no-cpu-baseline --no-extra > gpurun_out/ab/abl_${abl}_$r.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/ab/abl_${abl}_$r.json')); k=d['kernel_ms']
print('abl=$abl', $r, f\"{d['ms_per_step']:.3f} ms/step\", ' '.join(f'{n}={v:.3f}' for n, v in sorted(k.items())))
" >> gpurun_out/ab/summary_abl.txt
done; done
