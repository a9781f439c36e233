# fp8 wgrad fix check; persistent GEMM (incremental cursor) K-scan with/without start stagger;
# tests; same-box A/B (A base lib, B new); c5 fp8 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/ab
rm -f gpurun_out/ab/summary3.txt gpurun_out/ab/summary_c5f8.txt
timeout -k 10 200 python -u tools/dbg_fp8w.py > gpurun_out/dbg_fp8w.txt 2>&1
(MLVAE_GEMM_STAGGER=0 GEMM_VARS=0 GEMM_EPIS=16 timeout -k 10 120 python -u tools/gemm_kscan.py || exit 1; for abl in 0 40976 20496; do MLVAE_GEMM_ABL=$abl GEMM_VARS=0 GEMM_EPIS=16 timeout -k 10 120 python -u tools/gemm_kscan.py || exit 1; done; GEMM_VARS=12 GEMM_EPIS=16 timeout -k 10 120 python -u tools/gemm_kscan.py) > gpurun_out/gemm_kscan_r4m.txt 2>&1 && \
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gemm_fast.py tests/test_gpu_fp8.py tests/test_gpu_parity_bench.py > gpurun_out/r4m_tests.log 2>&1 && \
KNOB=0 CFGS="c3 c2 c5bf16" bash tools/gpu_ab3.sh && mv gpurun_out/ab/summary3.txt gpurun_out/ab/summary_r4m.txt && \
for r in 1 2; do
  for v in A B C; do
    if [ $v = A ]; then E=0; c=c5; elif [ $v = B ]; then E=1; c=c5; else E=1; c=c5bf16; fi
    MLVAE_FP8_WGRAD=$E timeout -k 10 150 python -u bench.py --config $c --no-cpu-baseline --no-extra > gpurun_out/ab/f8_${v}_$r.json 2> gpurun_out/ab/f8_${v}_$r.err || exit 1
    python3 -c "
import json
d=json.load(open('gpurun_out/ab/f8_${v}_$r.json')); k=d['kernel_ms']
print('$v', '$c', 'wgrad8=$E', $r, f\"{d['ms_per_step']:.3f} ms/step\", ' '.join(f'{n}={v:.3f}' for n, v in sorted(k.items())))
" >> gpurun_out/ab/summary_c5f8.txt
  done
done
