set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
rm -f gpurun_out/ab/summary3.txt
KNOB=536871008 CFGS="c3 c5bf16" bash tools/gpu_ab3.sh && mv gpurun_out/ab/summary3.txt gpurun_out/ab/summary_stagger3.txt && \
KNOB=536870976 CFGS="c3 c2" bash tools/gpu_ab3.sh && mv gpurun_out/ab/summary3.txt gpurun_out/ab/summary_stagger2.txt
