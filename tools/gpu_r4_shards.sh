# per-GPU shards of the metric's B=256 with the final code, one box: B=256 / 128 / 64 / 32
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/shards
for c in c3 c3h c5bf16 c2; do
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --no-extra > gpurun_out/shards/r04_$c.json 2>/dev/null || exit 1
done
