# round-end record: GPU tests + smoke + bench (with cpu_baseline), then the rocprofv3 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh && bash tools/gpu_profile.sh
