# layer-0 h written pre-shifted (mlvae_lstm_fwd_z2 y_bf16_prev): the fused-z forward tests, the
# c3 / c5 step parity tests, then c3 and c5 benches and a c3 kernel trace (dW_hh_l0 on VAR 18)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
OUT=gpurun_out/ybp
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_lstm_wide.py tests/test_gpu_parity_bench.py tests/test_gpu_step_parity.py \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
grep -E "passed|failed|^\[c|^\[fp8" $OUT/pytest.log | tail -12
REPS=2 bash tools/gpu_run.sh - "c3 c5 c2" ybpab "MLVAE_NONE=0" "MLVAE_NONE=1" || exit 1
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o c3 -- \
  python3 -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-extra > $OUT/trace.log 2>&1
