# same-box sweep of an environment knob over bench runs: bash tools/gpu_knob.sh VAR v1 v2 ...
# (two alternating rounds; one log per run under gpurun_out/knob_<VAR>_<v>_<round>.log)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
VAR=$1; shift
for r in 1 2; do
  for v in "$@"; do
    ( export "$VAR=$v"; timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 30 > gpurun_out/knob_${VAR}_${v}_$r.log 2>&1 ) || exit 1
  done
done
