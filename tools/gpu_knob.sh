# same-box sweep of environment knobs over bench runs (two alternating rounds):
#   bash tools/gpu_knob.sh "<bench args>" "VAR=v1 VAR2=w1" "VAR=v2" ...
# one log per setting and round under gpurun_out/knob/<i>_<round>.log
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/knob
ARGS=$1; shift
for r in 1 2; do
  i=0
  for setting in "$@"; do
    ( export $setting; timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extra $ARGS > gpurun_out/knob/${i}_$r.log 2>&1 ) || exit 1
    echo "$setting" > gpurun_out/knob/${i}.name
    i=$((i+1))
  done
done
