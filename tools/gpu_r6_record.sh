# round-6 record: GPU tests + smoke + bench (cpu_baseline included), the trajectory printouts
# (-s, both teacher-forced modes and the free-running fp64-anchored run), then rocprofv3 stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
bash tools/gpu_check.sh && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_trajectory.py -m gpu -x -v -s --timeout 240 --timeout-method thread \
  -k "teacher_forced or free_running" > gpurun_out/trajectory.log 2>&1 && \
bash tools/gpu_profile.sh
