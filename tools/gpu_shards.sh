# per-GPU shard step times of the metric's B=256 at N = 1/2/4/8 (c3, c3h, c5bf16, c2) on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/shards
for c in c3 c3h c5bf16 c2; do
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --no-extra > gpurun_out/shards/$c.log 2>&1 || exit 1
done
