# HBM traffic per kernel: two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over a
# short bench run of config $1 (default c3), merged into gpurun_out/pmc/pmc_traffic.json under that
# config's name (tools/pmc_summary.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/pmc
CFG=${1:-c3}
[ -f profiles/pmc_traffic.json ] && [ ! -f gpurun_out/pmc/pmc_traffic.json ] && cp profiles/pmc_traffic.json gpurun_out/pmc/
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o fetch -- \
  python3 -u bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/pmc/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o write -- \
  python3 -u bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/pmc/write.log 2>&1 && \
python3 tools/pmc_summary.py gpurun_out/pmc/fetch_counter_collection.csv \
  gpurun_out/pmc/write_counter_collection.csv gpurun_out/pmc/pmc_traffic.json $CFG
