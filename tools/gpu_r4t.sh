# c3 step with the GEMM tile-order group 8 vs 4 (alternating, same box); c3h (B=128) shard;
# c4 kernel stats (conv breakdown)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/ab gpurun_out/prof_c4b
rm -f gpurun_out/ab/summary_gm.txt
for r in 1 2 3; do for gm in 4 8; do
  MLVAE_GEMM_GROUP_M=$gm timeout -k 10 150 python -u bench.py --config c3 --no-cpu-baseline --no-extra > gpurun_out/ab/gm_${gm}_$r.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/ab/gm_${gm}_$r.json')); k=d['kernel_ms']
print('group_m=$gm', $r, f\"{d['ms_per_step']:.3f} ms/step\", ' '.join(f'{n}={v:.3f}' for n, v in sorted(k.items())))
" >> gpurun_out/ab/summary_gm.txt
done; done && \
timeout -k 10 150 python -u bench.py --config c3h --no-cpu-baseline --no-extra > gpurun_out/ab/c3h.json 2>/dev/null && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4b -o run -- python3 -u bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/prof_c4b/bench.log 2>&1
