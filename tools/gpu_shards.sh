# per-GPU shards of the metric's B=256 (N = 1/2/4/8 -> B = 256/128/64/32), one box, final code
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/shards
for c in c3 c3h c5bf16 c2; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-extra > gpurun_out/shards/r06_$c.json 2> gpurun_out/shards/r06_$c.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/shards/r06_$c.json').read().strip().splitlines()[-1]); print('$c', round(d['ms_per_step'],3), {k: round(x,3) for k,x in d.get('kernel_ms',{}).items()})"
done
