# knob sweep over two bench configs (c3 then c2): bash tools/gpu_knob2.sh "<settings...>"
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_knob.sh "--config c3" "$@" && mkdir -p gpurun_out/knob_c3 && mv gpurun_out/knob/* gpurun_out/knob_c3/ && \
bash tools/gpu_knob.sh "--config c2" "$@" && mkdir -p gpurun_out/knob_c2 && mv gpurun_out/knob/* gpurun_out/knob_c2/
