# fp8 delayed scales at the step start (side stream) vs before each BPTT: fp8 parity tests, then
# same-process A/B at c5
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
OUT=gpurun_out/f8early
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fp8.py tests/test_gpu_parity_bench.py -k "fp8 or c5" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
grep -E "passed|failed|step 2" $OUT/pytest.log | tail -4
timeout -k 10 400 python -u tools/step_ab.py c5 "" "f8_early=False" > $OUT/ab_c5.txt 2>&1 || { tail -5 $OUT/ab_c5.txt; exit 1; }
tail -2 $OUT/ab_c5.txt
