# host-side issue overhead probe (c3, c2), then the round-end rocprofv3 kernel stats of the c3 bench
# and the two PMC passes (FETCH_SIZE, WRITE_SIZE)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 180 python -u tools/cpu_overhead.py c3 > gpurun_out/cpu_overhead.txt 2>&1 && \
timeout -k 10 180 python -u tools/cpu_overhead.py c2 >> gpurun_out/cpu_overhead.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/prof/bench.log 2>&1 && \
bash tools/gpu_pmc.sh c3
