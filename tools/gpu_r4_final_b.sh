# round-end record, part 2: rocprofv3 kernel stats of the c3 bench (20 timed steps) and the two
# PMC passes (FETCH_SIZE, WRITE_SIZE) for the HBM traffic of c3's kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/prof/bench.log 2>&1 && \
bash tools/gpu_pmc.sh c3
