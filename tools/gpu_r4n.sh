# conv (2-stage slab reduce, dgrad aux with the window) + fp8 weight gradient + VAR 12 default again:
# tests, c4 A/B (A base lib, B new), c5 fp8 vs bf16 alternating, c4 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/ab gpurun_out/prof_c4
rm -f gpurun_out/ab/summary3.txt gpurun_out/ab/summary_c5f8.txt
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_fp8.py tests/test_gpu_parity_bench.py > gpurun_out/r4n_tests.log 2>&1 && \
KNOB=0 CFGS="c4" bash tools/gpu_ab3.sh && mv gpurun_out/ab/summary3.txt gpurun_out/ab/summary_r4n_c4.txt && \
for r in 1 2 3; do
  for c in c5 c5bf16; do
    timeout -k 10 150 python -u bench.py --config $c --no-cpu-baseline --no-extra > gpurun_out/ab/f8n_${c}_$r.json 2> gpurun_out/ab/f8n_${c}_$r.err || exit 1
    python3 -c "
import json
d=json.load(open('gpurun_out/ab/f8n_${c}_$r.json')); k=d['kernel_ms']
print('$c', $r, f\"{d['ms_per_step']:.3f} ms/step\", ' '.join(f'{n}={v:.3f}' for n, v in sorted(k.items())))
" >> gpurun_out/ab/summary_c5f8.txt
  done
done && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o run -- python3 -u bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/prof_c4/bench.log 2>&1
