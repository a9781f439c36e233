# fp8 recurrence (F8R) + conv slab layout + nt epilogue stores: tests (parity printed, not -x),
# K-scan nt A/B, c5 fp8 rec8 on/off vs bf16, c4 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/ab
rm -f gpurun_out/ab/summary3.txt gpurun_out/ab/summary_c5r8.txt gpurun_out/ab/summary_abl.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_lstm_wide.py > gpurun_out/r4p_tests.log 2>&1 && \
timeout -k 10 400 python -u -m pytest -q -s --timeout 200 --timeout-method thread tests/test_gpu_fp8.py tests/test_gpu_parity_bench.py -k "fp8 or c5" > gpurun_out/r4p_fp8.log 2>&1
rc=$?; if [ $rc -gt 1 ]; then echo "fp8 tests ended with $rc: stopping" >> gpurun_out/r4p_fp8.log; exit $rc; fi
(for abl in 0 32; do MLVAE_GEMM_ABL=$abl GEMM_VARS=12 GEMM_EPIS=16,0 timeout -k 10 120 python -u tools/gemm_kscan.py || exit 1; done) > gpurun_out/gemm_kscan_r4p.txt 2>&1 && \
for r in 1 2; do
  for v in A B C; do
    if [ $v = A ]; then E=1; c=c5; elif [ $v = B ]; then E=0; c=c5; else E=1; c=c5bf16; fi
    MLVAE_FP8_REC=$E timeout -k 10 150 python -u bench.py --config $c --no-cpu-baseline --no-extra > gpurun_out/ab/r8_${v}_$r.json 2> gpurun_out/ab/r8_${v}_$r.err || exit 1
    python3 -c "
import json
d=json.load(open('gpurun_out/ab/r8_${v}_$r.json')); k=d['kernel_ms']
print('$v', '$c', 'rec8=$E', $r, f\"{d['ms_per_step']:.3f} ms/step\", ' '.join(f'{n}={v:.3f}' for n, v in sorted(k.items())))
" >> gpurun_out/ab/summary_c5r8.txt
  done
done && \
for r in 1 2; do for abl in 0 32; do
  MLVAE_GEMM_ABL=$abl timeout -k 10 150 python -u bench.py --config c3 --no-cpu-baseline --no-extra > gpurun_out/ab/abl_${abl}_$r.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/ab/abl_${abl}_$r.json')); k=d['kernel_ms']
print('abl=$abl', $r, f\"{d['ms_per_step']:.3f} ms/step\", ' '.join(f'{n}={v:.3f}' for n, v in sorted(k.items())))
" >> gpurun_out/ab/summary_abl.txt
done; done && \
KNOB=0 CFGS="c4" bash tools/gpu_ab3.sh && mv gpurun_out/ab/summary3.txt gpurun_out/ab/summary_r4p_c4.txt
