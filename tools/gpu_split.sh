# split-K workgroup targets of the side-stream weight gradients (engine split_overlap / split_tail),
# same-process A/B at the shard configs
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
OUT=gpurun_out/split2
mkdir -p $OUT
for c in c5 c2 c5bf16; do
  timeout -k 10 400 python -u tools/step_ab.py $c "" "split_overlap=64" "split_overlap=32" "split_overlap=48" "split_overlap=64,split_tail=256" > $OUT/ab_$c.txt 2>&1 || { tail -5 $OUT/ab_$c.txt; exit 1; }
  tail -5 $OUT/ab_$c.txt
done
