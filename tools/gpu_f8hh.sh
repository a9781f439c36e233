# fp8 dW_hh (time-shifted rows in the fp8 TN kernel; the fp8 BPTT writes the e4m3 dG alone): the
# fp8 kernel tests, the c5 / fp8 step parity tests, the BPTT rerun test, then c5 fp8 vs bf16 steps
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
OUT=gpurun_out/f8hh
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fp8.py \
  tests/test_gpu_parity_bench.py -k "fp8 or c5" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
grep -E "passed|failed|\[c5|\[fp8|fp8 weight|c5 fp8|fp8 L=3" $OUT/pytest.log | tail -20
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_lstm_wide.py -k "rerun or bit" > $OUT/pytest_bptt.log 2>&1 || { tail -30 $OUT/pytest_bptt.log; exit 1; }
tail -1 $OUT/pytest_bptt.log
REPS=2 bash tools/gpu_run.sh - "c5 c5bf16" f8hhab "MLVAE_NONE=0" "MLVAE_NONE=1"
