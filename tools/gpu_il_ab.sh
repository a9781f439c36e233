set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
bash tools/gpu_round.sh || exit 1
for i in 1 2; do
 for il in 0 1; do
  MLVAE_WIDE_IL=$il timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-extra > gpurun_out/il${il}_c3_$i.log 2>&1 || exit 1
  MLVAE_WIDE_IL=$il timeout -k 10 120 python -u bench.py --config c2 --no-cpu-baseline --no-extra > gpurun_out/il${il}_c2_$i.log 2>&1 || exit 1
 done
done
