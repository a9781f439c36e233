# fp8 weight gradient (VAR 9): kernel tests, the fp8 step parity, then same-box c5 A/B:
# A = fp8 mode without the fp8 wgrad, B = fp8 mode (default), C = the bf16 step
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fp8.py > gpurun_out/r4k_tests.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_gpu_parity_bench.py -k c5 > gpurun_out/r4k_parity.log 2>&1 && \
rm -f gpurun_out/ab/summary_c5f8.txt && \
for r in 1 2 3; do
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
