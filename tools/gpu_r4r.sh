# the committed state vs the previous commit's library (A): c3 / c2 / c5bf16; C = the forward's
# s_sleep 1 retry back-off at full chip (debug bit 30)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/ab
rm -f gpurun_out/ab/summary3.txt
KNOB=1073741824 CFGS="c3 c2 c5bf16" bash tools/gpu_ab3.sh && mv gpurun_out/ab/summary3.txt gpurun_out/ab/summary_r4r.txt
