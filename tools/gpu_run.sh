# One gpurun session: a pytest selection, then bench configs, each GPU step under its own limit.
#   bash tools/gpu_run.sh "<pytest args | ->" "<bench configs | ->" <tag> ["<env A>" "<env B>" ...]
# With env variants (e.g. "MLVAE_LSTM_DBG=0" "MLVAE_LSTM_DBG=2048") every config is run twice per
# variant, alternating (same-box A/B); results in gpurun_out/<tag>/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
PYT=$1; CFGS=$2; TAG=${3:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
shift 3
VARS=("$@")
REPS=${REPS:-2}
[ ${#VARS[@]} -eq 0 ] && { VARS=("MLVAE_NONE=0"); REPS=1; }
if [ "$PYT" != "-" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $PYT \
    > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
fi
if [ "$CFGS" != "-" ]; then
  for c in $CFGS; do
    for r in $(seq $REPS); do
      for i in "${!VARS[@]}"; do
        f=$OUT/bench_${c}_v${i}_r${r}.json
        env ${VARS[$i]} timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-extra > $f 2> $f.err || exit $?
        python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$c', '${VARS[$i]}', 'r$r', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d.get('kernel_ms',{}).items()})"
      done
    done
  done
fi
