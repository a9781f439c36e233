# the batch / fp8-scaled side-stream split target (default) against the former fixed 128
# (split_overlap=256 reproduces it at B = 32 bf16 and B = 64 fp8), same process
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
OUT=gpurun_out/split3
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity_bench.py -k "c5 or fp8" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for c in c5 c2; do
  timeout -k 10 400 python -u tools/step_ab.py $c "" "split_overlap=256" > $OUT/ab_$c.txt 2>&1 || { tail -5 $OUT/ab_$c.txt; exit 1; }
  tail -2 $OUT/ab_$c.txt
done
