# rocprofv3 kernel stats under each MLVAE_LSTM_DBG setting (same box): bash tools/gpu_prof_ab.sh "<bench args>" v1 v2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
ARGS=$1; shift
for v in "$@"; do
  mkdir -p gpurun_out/profab/$v
  MLVAE_LSTM_DBG=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profab/$v -o run -- \
    python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra $ARGS > gpurun_out/profab/$v/bench.log 2>&1 || exit 1
done
