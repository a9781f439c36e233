# dW_hh as unshifted products minus the utterance-boundary terms: step parity tests, then
# same-process A/B of the engine attribute (tools/step_ab.py) at c3 / c2 / c4
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
OUT=gpurun_out/whh
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity_bench.py tests/test_gpu_step_parity.py tests/test_gpu_trajectory.py \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
grep -E "passed|failed|^\[c" $OUT/pytest.log | tail -8
for c in c3 c2 c4; do
  timeout -k 10 300 python -u tools/step_ab.py $c "" "whh_unshift=False" "whh_unshift=False,yb_prev=False" > $OUT/ab_$c.txt 2>&1 || { tail -5 $OUT/ab_$c.txt; exit 1; }
  tail -3 $OUT/ab_$c.txt
done
