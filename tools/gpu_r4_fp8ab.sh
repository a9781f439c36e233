# c5 shard fp8 vs bf16 with the final code, same box, alternating x3
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/ab
rm -f gpurun_out/ab/summary_fp8ab.txt
for r in 1 2 3; do for c in c5 c5bf16; do
  timeout -k 10 150 python -u bench.py --config $c --no-cpu-baseline --no-extra > gpurun_out/ab/fp8ab_${c}_$r.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/ab/fp8ab_${c}_$r.json')); k=d['kernel_ms']
print('$c', $r, f\"{d['ms_per_step']:.3f} ms/step\", ' '.join(f'{n}={v:.3f}' for n, v in sorted(k.items()) if n in ('proj_l1','dgrad_l1','lstm_fwd','lstm_bwd')))
" >> gpurun_out/ab/summary_fp8ab.txt
done; done
