# Average shader clock per kernel = GRBM_GUI_ACTIVE cycles / kernel duration, per debug mode:
#   bash tools/clock_pmc.sh <config> <mode> [<mode> ...]   -> gpurun_out/clk/<config>_<mode>_{pmc,trace}*
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/clk
CFG=$1; shift
for m in "$@"; do
  MLVAE_LSTM_DEBUG_MODE=$m timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/clk -o ${CFG}_${m}_pmc -- \
    python3 -u bench.py --config $CFG --steps 6 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/clk/${CFG}_${m}_pmc.log 2>&1 || exit 1
  MLVAE_LSTM_DEBUG_MODE=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/clk -o ${CFG}_${m}_trace -- \
    python3 -u bench.py --config $CFG --steps 6 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/clk/${CFG}_${m}_trace.log 2>&1 || exit 1
done
