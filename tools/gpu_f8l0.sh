# fp8 mode, e4m3 dG of both layers (layer 0: skinny e4m3 kernels + fp8 dW_hh_l0): fp8 kernel tests,
# the c5 / fp8 step parity tests, then c5 fp8 vs bf16 steps alternating, and a c5 kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
OUT=gpurun_out/f8l0
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fp8.py \
  tests/test_gpu_parity_bench.py -k "fp8 or c5" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
grep -E "passed|failed|\[c5|\[fp8|e4m3-operand|c5 fp8|fp8 L=3" $OUT/pytest.log | tail -20
REPS=2 bash tools/gpu_run.sh - "c5 c5bf16" f8l0ab "MLVAE_NONE=0" "MLVAE_NONE=1" || exit 1
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o c5 -- \
  python3 -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-extra > $OUT/trace.log 2>&1
