# c5 per-GPU shard: fp8 vs bf16, alternating rounds (same box)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/c5ab
for r in 1 2; do
  for c in c5 c5bf16; do
    timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --no-extra > gpurun_out/c5ab/${c}_$r.log 2>&1 || exit 1
  done
done
