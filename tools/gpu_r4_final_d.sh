# round-end record (after the fused layer-0 dZ / dW pass): every GPU test, smoke, the default bench
# line, then the c3 rocprofv3 kernel stats and the two PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 780 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 240 python -u bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/prof/bench.log 2>&1 && \
bash tools/gpu_pmc.sh c3
