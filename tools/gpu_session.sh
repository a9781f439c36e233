# One GPU session: pytest on the given test files (-m gpu), then a bench run.
#   bash tools/gpu_session.sh "<test files or -k expr>" "<bench.py args>" [tag]
# Logs under gpurun_out/<tag>/.  Every GPU step has its own time limit; a failed or
# timed-out step ends the session (no further GPU work after a fault).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
TAG=${3:-s}
mkdir -p gpurun_out/$TAG
if [ -n "$1" ]; then
  timeout -k 10 600 python -u -m pytest $1 -v -s --timeout 240 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -n "$2" ]; then
  timeout -k 10 400 python -u bench.py $2 > gpurun_out/$TAG/bench.log 2>&1
  echo "bench rc=$?"
fi
