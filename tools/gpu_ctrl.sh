# control: the fe3633f snapshot (scratch/fe36: its engine, bench and library) against the current
# tree, c3 alternating on one box (+ the wide-recurrence tests first)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
OUT=gpurun_out/ctrl2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_lstm_wide.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do
  for c in c3; do
    (cd scratch/fe36 && timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-extra > ../../$OUT/old_${c}_$r.json 2> ../../$OUT/old_${c}_$r.err) || exit 1
    timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-extra > $OUT/new_${c}_$r.json 2> $OUT/new_${c}_$r.err || exit 1
    for v in old new; do
      python3 -c "import json; d=json.loads(open('$OUT/${v}_${c}_$r.json').read().strip().splitlines()[-1]); print('$v', '$c', $r, round(d['ms_per_step'],3), {k: round(x,3) for k,x in d.get('kernel_ms',{}).items()})"
    done
  done
done
