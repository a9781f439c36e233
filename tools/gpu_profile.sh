# bench + rocprofv3 kernel trace/stats of the default bench command (c2, bf16); outputs under gpurun_out/prof
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/prof
timeout -k 10 120 python -u bench.py --no-cpu-baseline > gpurun_out/prof/bench_plain.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof/bench.log 2>&1
